"""Headline benchmark: ResNet-50 synthetic DDP training on MI355X with the
libgsync gradient-sync engine (BASELINE.json metric "images/sec (node)
ResNet-50 at 1/2/4/8 MI355X; grad-sync bus GB/s").

One step = forward (bf16 autocast, channels_last) + backward with the
libgsync bucketer packing/all-reducing/unpacking buckets on its own RCCL
stream under backward + fused SGD-momentum/WD update, on 256 synthetic
224x224 images per GPU generated on the device once (inputs resident in HBM).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
`roofline` for the dominant grad-sync kernel (the fused SGD update:
20 B/param algorithmic, timed with HIP events on the stream it runs on),
`grad_sync` (RCCL bus bandwidth of the bucket all-reduces, events on the
libgsync comm stream, against (n-1) x 153 GB/s xGMI) and `cpu_baseline`
(the reference's torch-DDP/gloo path on the host cores, rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

T_START = time.time()  # --wall-budget-s counts from here (covers warm-up's MIOpen compiles)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
HBM_COPY_GBPS = 6290.0  # MI355X_MICROARCH.md's measured float4 copy ceiling (report both)
XGMI_LINK_GBPS = 153.0  # per point-to-point link; bus roofline (n-1) x 153


def _host_cores() -> dict:
    """The host cores this process may use: its CPU affinity, capped by the
    cgroup's CPU quota when one is set (a GPU box's share of a larger machine —
    os.cpu_count() reports the whole machine there)."""
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = int(parts[0]) / int(f.read().split()[0])
            if quota is not None:
                break
        except (OSError, ValueError, IndexError, ZeroDivisionError):
            continue
    used = max(1, min(affinity, int(quota)) if quota else affinity)
    return {"cores_used": used, "affinity": affinity, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "rule": "min(CPU affinity, cgroup CPU quota); the torch DDP/gloo ranks split them, cores // ws each"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50", choices=["resnet18", "resnet50", "resnet152"])
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--bucket-cap-mb", type=float, default=None)
    ap.add_argument("--bucket-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam"])
    ap.add_argument("--engine", default="ddp", choices=["ddp", "zero1", "zero2", "colossal"],
                    help="ddp = headline (BASELINE configs[1-2]); zero1/zero2 = DeepSpeed-style (configs[3]); "
                         "colossal = the Colossal Booster shim as run.sh drives it (TorchDDPPlugin, fp16 mixed "
                         "precision, HybridAdam; configs[4] with --model resnet152)")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--grad-as-bucket-view", action="store_true",
                    help="DDP(gradient_as_bucket_view=True): grads alias the buckets, no unpack pass")
    # MIOpen Find (benchmark=1) tunes every conv for minutes on a fresh box; the
    # immediate-mode solutions are what the 5.9k img/s number was measured with
    ap.add_argument("--cudnn-benchmark", type=int, default=0)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU/gloo reference path (rank 0, N=1)")
    ap.add_argument("--collective-bench", type=int, default=-1,
                    help="standalone RCCL timing of the step's collectives after the timed region "
                         "(-1: only when N > 1)")
    ap.add_argument("--pg-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: N>1 control-flow rehearsal with ranks sharing GPUs (not a measurement)")
    ap.add_argument("--impl", default="libgsync", choices=["libgsync", "torch"],
                    help="torch = the reference path on the same GPU (torch DDP + torch.optim SGD/Adam foreach; "
                         "with --engine colossal: + fp16 autocast, torch.amp.GradScaler, fused AdamW), for comparison")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: record the whole step (forward, backward + bucket sync, update) into one hipGraph "
                         "(CapturedStep, capturable optimizer) and replay it")
    ap.add_argument("--bucket-policy", default="torch", choices=["torch", "xgmi"],
                    help="DDP bucket caps: torch's (default, torch-parity layout) or from the live all-reduce "
                         "curve at N>1 (distributed_training_amd.ddp.xgmi_bucket_caps)")
    ap.add_argument("--last-bucket-cap-mb", type=float, default=None,
                    help="cap the last bucket in gradient-ready order (the exposed end-of-backward chain)")
    ap.add_argument("--zero-leg", type=int, default=1,
                    help="after the headline: BASELINE configs[3] (ZeRO-2, bf16 ResNet-50) timed on the same "
                         "ranks, reported as the line's `zero2` object (DDP engine; 0: off)")
    ap.add_argument("--colossal-leg", type=int, default=1,
                    help="after the headline: BASELINE configs[4] (Colossal shim, ResNet-152 fp32 grads, fp16 "
                         "autocast, HybridAdam, 128 img/GPU) on the same ranks, the line's `colossal` object "
                         "(DDP engine; 0: off)")
    ap.add_argument("--wall-budget-s", type=float, default=540.0,
                    help="whole-run wall budget from process start (warm-up compiles included): an optional leg "
                         "after the timed region runs only if its cost estimate (LEG_COST_S, measured) fits what "
                         "is left, else it is recorded as skipped; a leg still running past the budget ends "
                         "every rank after the line is printed, exit status 3 (0 = no budget)")
    ap.add_argument("--parity", type=int, default=1,
                    help="after the timed region: one self-checked step (distributed_training_amd.parity)")
    ap.add_argument("--kernel-rates", type=int, default=1,
                    help="after the timed region: every grad-sync kernel alone on this model's params (rank 0)")
    ap.add_argument("--optimizer-overlap", type=int, default=0,
                    help="1: DDP._register_fused_optim — each bucket's fused update runs behind its unpack "
                         "under backward (torch's overlapped-optimizer API); no optimizer.step() after backward")
    ap.add_argument("--policy-ab", type=int, default=-1,
                    help="after the timed region: re-wrap the model with each DDP bucket policy (torch, xgmi, "
                         "last-bucket cap 1 MiB, torch again) and time each, with tail, bus bandwidth and parity "
                         "(-1: only at N > 1 on the DDP engine) — the data for DESIGN §8's policy rule")
    ap.add_argument("--torch-leg", type=int, default=1,
                    help="after the legs: the reference's own GPU path (torch DDP + torch.optim.SGD foreach) on the "
                         "same model / batch / step, timed like the headline; vs_baseline = libgsync / it; "
                         "and configs[4] on torch beside the colossal leg (0: off)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def collective_bench(ddp, zero, world, iters=10, warmup=3):
    """The step's collectives alone (after the timed region, every rank): each
    bucket's all-reduce (DDP) or reduce-scatter + all-gather (ZeRO), back to back
    on libgsync's comm stream, HIP events around each, after a barrier.
    busBW = S/t x 2(n-1)/n (all-reduce), S/t x (n-1)/n (RS / AG), S = full buffer
    bytes, against the xGMI roofline (n-1) x 153 GB/s."""
    comm = ddp._comm if zero is None else zero._comm
    if comm is None:
        return None
    ops = []
    if zero is None:
        for b in ddp._bucketer.buffers:
            ops.append(("all_reduce", b.numel() * b.element_size(), lambda b=b: comm.all_reduce(b)))
        # the whole gradient as one message: the size-limited ceiling of the same link set
        whole = torch.zeros(sum(b.numel() for b in ddp._bucketer.buffers), dtype=ddp._bucketer.buffers[0].dtype,
                            device=ddp._bucketer.buffers[0].device)
        ops.append(("all_reduce_whole_grad", whole.numel() * whole.element_size(), lambda: comm.all_reduce(whole)))
        # message-size curve of the same link set, for the bucket-size choice (bucket_cap_mb)
        for mb in (1, 4, 16, 64):
            buf = torch.zeros(mb * 1024 * 1024 // 4, dtype=torch.float32, device=whole.device)
            ops.append((f"all_reduce_{mb}MiB", buf.numel() * 4, lambda buf=buf: comm.all_reduce(buf)))
    else:
        for g, sh in zip(zero.grad_bufs, zero.grad_shards):
            if zero.stage == 2:
                ops.append(("reduce_scatter", g.numel() * g.element_size(),
                            lambda g=g, sh=sh: comm.reduce_scatter(g, sh)))
            else:
                ops.append(("all_reduce", g.numel() * g.element_size(), lambda g=g: comm.all_reduce(g)))
        for flat, shard in zip(zero.param_flats, zero.param_shards):
            ops.append(("all_gather", flat.numel() * flat.element_size(),
                        lambda f=flat, s=shard: comm.all_gather(s, f)))
    out = []
    torch.cuda.synchronize()
    _BenchColl(comm, comm.device, "nccl").barrier()
    with torch.cuda.stream(comm.stream):
        for kind, nbytes, fn in ops:
            for _ in range(warmup):
                fn()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
            for a, b in evs:
                a.record()
                fn()
                b.record()
            out.append((kind, nbytes, evs))
    torch.cuda.synchronize()
    rows, tot_ms, tot_bus_bytes = [], 0.0, 0.0
    peak = (world - 1) * XGMI_LINK_GBPS
    for kind, nbytes, evs in out:
        ms = sorted(a.elapsed_time(b) for a, b in evs)[len(evs) // 2]
        f = 2 * (world - 1) / world if kind.startswith("all_reduce") else (world - 1) / world
        bus = nbytes / (ms * 1e-3) * f / 1e9
        rows.append({"op": kind, "bytes": nbytes, "median_ms": ms, "algbw_GBps": nbytes / (ms * 1e-3) / 1e9,
                     "bus_GBps": bus, "frac": (bus / peak) if peak > 0 else None})
        if kind in ("all_reduce", "reduce_scatter", "all_gather"):  # the step's own collectives only
            tot_ms += ms
            tot_bus_bytes += nbytes * f
    agg = tot_bus_bytes / (tot_ms * 1e-3) / 1e9
    return {"per_op": rows, "ms_per_step": tot_ms, "bus_GBps": agg, "xgmi_peak_GBps": peak,
            "frac": (agg / peak) if peak > 0 else None,
            "timing": "HIP events on libgsync's comm stream, median of 10 after 3 warmup, ops back to back"}


def _kernel_rows(shapes, dev, iters, shapes16=None):
    """Every grad-sync kernel of the step on one parameter set (shapes), warm and
    alone on the GPU: pack fp32 x1/ws, pack to bf16, unpack (+ fused Σg²), Σg² on
    a bucket-layout plan (64-element alignment, as the DDP buckets), the update
    kernels on an update plan (as FusedSGD / FusedAdam build it).  Algorithmic
    bytes / average per call (plan launch timer: HIP events on the launch stream
    around each kernel, every launch of a multi-launch call counted)."""
    from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units

    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(7)
    grads = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    plan = TensorListPlan(numels, dev, align=64)
    plan.set_ptrs(1, grads)
    flat = torch.zeros(plan.flat_numel, device=dev)
    flat16 = torch.zeros(plan.flat_numel, device=dev, dtype=torch.bfloat16)
    sq = torch.zeros(1, device=dev)

    def rate(fn, p_):
        for _ in range(3):
            fn()
        p_.timer_enable(4 * iters)  # room for every launch of a multi-launch call (the ring keeps the last)
        for _ in range(iters):
            fn()
        ts = p_.timer_read()
        p_.timer_enable(0)
        return sum(ts) / iters  # per call: every launch the call makes counts

    rows = {}
    for name, nbytes, fn in (
            ("pack_f32", 8 * n, lambda: plan.pack(1, torch.float32, flat, 0.125, 1)),
            ("pack_f32_to_bf16", 6 * n, lambda: plan.pack(1, torch.float32, flat16, 0.125, 1)),
            ("unpack_f32", 8 * n, lambda: plan.unpack(flat, 1, torch.float32)),
            ("unpack_f32+sqnorm", 8 * n, lambda: plan.unpack(flat, 1, torch.float32, sqnorm=sq)),
            ("sqnorm_f32", 4 * n, lambda: plan.sqnorm(1, torch.float32, sq))):
        ms = rate(fn, plan)
        rows[name] = {"alg_bytes": nbytes, "avg_ms": ms, "GBps": nbytes / (ms * 1e-3) / 1e9}
    # Σg² as a clip after a libgsync DDP runs it: its first read of grads the unpack has
    # just written with non-temporal stores (per iteration: the unpack, then Σg²; the
    # Σg² launches alone timed), under the default load rule and the non-temporal hint
    # (gs_plan_set_read_hint) — the looped row above reads grads its own previous pass
    # left in the cache
    from distributed_training_amd import _lib as L

    for name, hint in (("sqnorm_f32_after_unpack", 0), ("sqnorm_f32_after_unpack_nt", 1)):
        plan.set_read_hint(hint)
        for _ in range(3):
            plan.unpack(flat, 1, torch.float32)
            plan.sqnorm(1, torch.float32, sq)
        plan.timer_enable(4 * iters)
        for _ in range(iters):
            plan.unpack(flat, 1, torch.float32)
            plan.sqnorm(1, torch.float32, sq)
        ms = sum(plan.timer_read_by_kind().get(L.GS_OP_SQNORM, [])) / iters
        plan.timer_enable(0)
        rows[name] = {"alg_bytes": 4 * n, "avg_ms": ms, "GBps": 4 * n / (ms * 1e-3) / 1e9,
                      "read_hint": "the size rule (cached below 256 MiB)" if hint == 0 else "non-temporal"}
    plan.set_read_hint(0)
    # the 16-bit bucket paths: ZeRO's bf16 grads -> bf16 bucket (configs[3]) and the bf16
    # bucket -> fp32 grads unpack (DDP bucket_dtype=bf16).  shapes16: their own (larger)
    # parameter set, so that a 16-bit source is past the Infinity Cache too
    if shapes16 is None:
        plan16, n16, g32, f16 = plan, n, grads, flat16
    else:
        del flat, flat16
        numels16 = [int(torch.Size(s_).numel()) for s_ in shapes16]
        n16 = sum(numels16)
        plan16 = TensorListPlan(numels16, dev, align=64)
        g32 = [torch.randn(s_, device=dev, generator=g) * 0.01 for s_ in shapes16]
        f16 = torch.zeros(plan16.flat_numel, device=dev, dtype=torch.bfloat16)
    grads16 = [gr.to(torch.bfloat16) for gr in g32]
    plan16.set_ptrs(1, grads16)
    ms = rate(lambda: plan16.pack(1, torch.bfloat16, f16, 0.125, 1), plan16)
    rows["pack_bf16"] = {"alg_bytes": 4 * n16, "avg_ms": ms, "GBps": 4 * n16 / (ms * 1e-3) / 1e9, "elems": n16}
    plan16.set_ptrs(1, g32)
    ms = rate(lambda: plan16.unpack(f16, 1, torch.float32), plan16)
    rows["unpack_bf16_to_f32"] = {"alg_bytes": 6 * n16, "avg_ms": ms, "GBps": 6 * n16 / (ms * 1e-3) / 1e9,
                                  "elems": n16}
    del f16, grads16, g32, plan16
    torch.cuda.empty_cache()
    up = TensorListPlan(numels, dev, task_units=update_task_units(dev))
    ps = [torch.randn(s, device=dev, generator=g) for s in shapes]
    bs = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    vs = [torch.rand(s, device=dev, generator=g) * 1e-4 for s in shapes]
    up.set_ptrs(0, ps)
    up.set_ptrs(1, grads)
    up.set_ptrs(2, bs)
    ms = rate(lambda: up.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False), up)
    rows["sgd_momentum_wd"] = {"alg_bytes": 20 * n, "avg_ms": ms, "GBps": 20 * n / (ms * 1e-3) / 1e9}
    # the clip path as the folded clip runs it (DeepSpeed gradient_clipping,
    # R:resnet/deepspeed/deepspeed_train.py:195): Σg² partial sums, then the update
    # whose workgroups form the coefficient from them — both launches timed
    ms = rate(lambda: up.sqnorm_partial(1, torch.float32), up)
    rows["sqnorm_partial_f32"] = {"alg_bytes": 4 * n, "avg_ms": ms, "GBps": 4 * n / (ms * 1e-3) / 1e9}
    clip_out = torch.zeros(3, device=dev)

    def clipped_sgd():
        up.sqnorm_partial(1, torch.float32)
        up.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)

    up.set_clip(1.0, 1e-6, None, out=clip_out)
    ms = rate(clipped_sgd, up)
    up.set_clip(None)
    rows["clip_path_sgd"] = {"alg_bytes": 24 * n, "avg_ms": ms, "GBps": 24 * n / (ms * 1e-3) / 1e9,
                             "launches": "sqnorm_partial + clipped sgd"}
    # clip_grad_norm_ as the drop-in runs it (T:nn/utils/clip_grad.py:165-174; the clip the
    # DeepSpeed config sets, R:resnet/deepspeed/deepspeed_train.py:195): the Σg² partial sums,
    # then the scale pass whose workgroups fold them (two launches, both timed); clipping
    # active (max_norm below ‖g‖: read 4 + read/write 8 B per element), the grads restored
    # by an untimed copy before each call
    from distributed_training_amd import optim as OPT

    cps = [torch.nn.Parameter(torch.empty(s, device=dev)) for s in shapes]
    cgs = [gr.clone() for gr in grads]
    for p_, g_ in zip(cps, cgs):
        p_.grad = g_
    OPT.clip_grad_norm_(cps, 1e-3)
    cplan = OPT._NORM_PLANS[tuple(numels) + (cgs[0].device,)]

    def clip_call():
        torch._foreach_copy_(cgs, grads)
        OPT.clip_grad_norm_(cps, 1e-3)

    ms = rate(clip_call, cplan)
    rows["clip_grad_norm"] = {"alg_bytes": 12 * n, "avg_ms": ms, "GBps": 12 * n / (ms * 1e-3) / 1e9,
                              "launches": "sqnorm_partial + clip_scale (the coefficient folded per workgroup)",
                              "restore": "an untimed copy of the grads before each call"}
    del cps, cgs
    up.set_ptrs(3, vs)
    ms = rate(lambda: up.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5), up)
    rows["adam"] = {"alg_bytes": 28 * n, "avg_ms": ms, "GBps": 28 * n / (ms * 1e-3) / 1e9}
    for r in rows.values():
        r["frac"] = r["GBps"] / HBM_PEAK_GBPS
    return n, rows


def zero_clip_path_rows(n_params, dev, comm, shard_world=8, iters=20):
    """configs[3]'s end-of-step clip path as its N>1 branch runs it (zero.py), on
    one rank's shard of an N=`shard_world` ZeRO-2 run (ResNet-50: 25.56 M / 8 ≈
    3.2 M elements; bf16 grads, fp32 master / exp_avg / exp_avg_sq, bf16 param
    write), every launch and the collective timed together (HIP events on the
    stream they run on), over the engine's RCCL communicator (one rank here):

    * ``clip_path_zero_n8``: Σg² partial sums of the shard (gs_sqnorm_partial_out:
      one per workgroup of a <= 1024-workgroup grid at this size, 780 floats, in
      a 1 Ki-float buffer) -> ONE SUM all-reduce of the buffer -> the AdamW update
      folding it
      (gs_plan_set_clip_groups) — the round-4/5 path;
    * ``clip_path_zero_n8_scalar``: round 3's form — Σg² with its in-kernel
      combine -> SUM all-reduce of the scalar -> the update (gs_plan_set_clip).

    Algorithmic bytes per element: Σg² 2 (bf16 read) + AdamW 28 (p r/w 8, g 2,
    m r/w 8, v r/w 8, bf16 param 2) = 30."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units

    q = shard_world * 64
    shard = (n_params + q - 1) // q * q // shard_world
    g = torch.Generator(device=dev).manual_seed(11)
    master = torch.randn(shard, device=dev, generator=g)
    grads = (torch.randn(shard, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    m = torch.randn(shard, device=dev, generator=g) * 1e-3
    v = torch.rand(shard, device=dev, generator=g) * 1e-6
    p16 = master.to(torch.bfloat16)
    plan = TensorListPlan([shard], dev, task_units=update_task_units(dev))
    for k, t in enumerate((master, grads, m, v, p16)):
        plan.set_ptrs(k, [t])
    groups = torch.zeros(L.GS_RED_PARTIALS, device=dev)
    sq = torch.zeros(1, device=dev)
    out = torch.zeros(3, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def adam():
        plan.adam(torch.bfloat16, 1e-3, 0.8, 0.999, 1e-8, 3e-7, True, False, -1e-3, 0.5, lowp_dtype=torch.bfloat16)

    # as zero.py since round 6: the all-reduce's watchdog mark rides on the update kernel
    # (gs_allreduce_marked), in both forms
    def folded():  # as zero.py: the whole partial-sum buffer travels and is folded
        plan.sqnorm_partial_out(1, torch.bfloat16, groups)
        comm.all_reduce(groups, stream=stream, consumer=plan.handle)
        plan.set_clip_groups(1.0, 1e-6, groups, groups.numel(), out=out)
        adam()

    def scalar():
        plan.sqnorm(1, torch.bfloat16, sq)
        comm.all_reduce(sq, stream=stream, consumer=plan.handle)
        plan.set_clip(1.0, 1e-6, sq, out=out)
        adam()

    # The step's end runs behind backward's queued kernels, so the host enqueues these
    # launches ahead of the GPU: time them the same way, behind a spin kernel long
    # enough for the host to queue every launch of the call (torch.cuda._sleep,
    # calibrated to ~150 µs), HIP events right around the call; the host-paced time
    # (no spin: each launch waits for its ctypes / RCCL enqueue) is reported beside it.
    spin = None
    if hasattr(torch.cuda, "_sleep"):
        a0, b0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        torch.cuda._sleep(1_000_000)
        b0.record()
        torch.cuda.synchronize()
        spin = max(1, int(1_000_000 * 0.15 / max(a0.elapsed_time(b0), 1e-3)))

    def window(fn, pre_spin):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in evs:
            if pre_spin:
                torch.cuda._sleep(spin)
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in evs) / iters

    rows = {}
    for name, fn in (("clip_path_zero_n8", folded), ("clip_path_zero_n8_scalar", scalar)):
        for _ in range(3):
            fn()
        host_ms = window(fn, False)
        ms = window(fn, True) if spin else host_ms
        plan.timer_enable(4 * iters)  # the kernels alone (plan launch timer), a separate pass
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        kern = plan.timer_read_by_kind()
        plan.timer_enable(0)
        nbytes = 30 * shard
        sq_ms = sum(kern.get(L.GS_OP_SQNORM, [])) / iters
        up_ms = sum(kern.get(L.GS_OP_ADAM, [])) / iters
        rows[name] = {"alg_bytes": nbytes, "avg_ms": ms, "GBps": nbytes / (ms * 1e-3) / 1e9,
                      "frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, "shard_elems": shard,
                      "kernels_ms": sq_ms + up_ms, "sqnorm_kernel_ms": sq_ms, "update_kernel_ms": up_ms,
                      "host_paced_ms": host_ms,
                      "timing": ("HIP events around the call, the stream pre-loaded by a spin kernel (the launches "
                                 "queued ahead, as behind backward)" if spin else "HIP events around the call"),
                      "launches": ("sqnorm_partial_out + all_reduce(partials) + clipped AdamW"
                                   if name == "clip_path_zero_n8" else
                                   "sqnorm (in-kernel combine) + all_reduce(scalar) + clipped AdamW"),
                      "watchdog_mark": "the all-reduce's, on the update kernel's stop event (gs_allreduce_marked)"}
    plan.set_clip(None)
    rows["clip_path_zero_n8"]["vs_scalar_form"] = (rows["clip_path_zero_n8_scalar"]["avg_ms"]
                                                   / rows["clip_path_zero_n8"]["avg_ms"])
    return rows


def _beyond_ic_shapes():
    """ResNet-152's parameter shapes twice: 120.4 M elements, a 481 MB gradient —
    every kernel's working set is well past the 256 MiB Infinity Cache."""
    from distributed_training_amd.resnet import MODELS

    with torch.device("meta"):
        m = MODELS["resnet152"](num_classes=1000)
    return [tuple(p.shape) for p in m.parameters()] * 2


def _beyond_ic_roofline(kernel_rates, zero, args, traffic_json):
    """The headline update kernel's true-HBM rate, measured in this run: the same
    kernel on the >256 MiB working set of grad_sync_kernel_rates (ResNet-152
    shapes x 2: 2.41 GB per SGD launch).  The in-step figure runs on ResNet-50's
    511 MB read/write set, partly served by the 256 MiB Infinity Cache right after
    the unpack wrote the grads (it reads above the measured copy ceiling), so the
    line's headline `frac` is this one; {} when the rows were
    not measured (the in-step figure then stays the headline, flagged)."""
    if not kernel_rates or zero is not None or args.engine != "ddp" or "beyond_ic" not in kernel_rates:
        return {}
    sgd = args.optimizer == "sgd"
    row = kernel_rates["beyond_ic"]["kernels"]["sgd_momentum_wd" if sgd else "adam"]
    traffic = None
    try:
        with open(traffic_json) as f:
            traffic = json.load(f).get(f"resnet152x2/{args.optimizer}", {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    out = {"achieved": row["GBps"], "frac": row["frac"], "avg_launch_ms": row["avg_ms"],
           "algorithmic_bytes_per_launch": row["alg_bytes"], "launches": kernel_rates.get("iters"),
           "traffic": traffic, "set": kernel_rates["beyond_ic"]["set"],
           "timing": "plan launch timer (hipExtLaunchKernel's events: the kernel's own start / end), "
                     "grad_sync_kernels.beyond_ic, after the timed region, back-to-back launches",
           "plain_stream_ceiling": _mix_ceiling("sgd3r2w" if sgd else "adam4r3w")}
    trace = _trace_check("SgdOp_beyond_ic" if sgd else "AdamOp_beyond_ic", row["alg_bytes"])
    if trace:
        out["rocprof"] = trace
    return out


def _trace_check(key, alg_bytes):
    """The same launches' average duration in the committed rocprofv3 kernel trace
    of the driver's command (profiles/trace_roofline.json, scripts/trace_bench.py)."""
    try:
        with open(os.path.join(REPO, "profiles", "trace_roofline.json")) as f:
            tr = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    if not tr:
        return None
    return {"kernel_trace_avg_ms": tr["avg_us"] * 1e-3, "launches": tr.get("timed_region_launches"),
            "frac_at_trace_duration": alg_bytes / (tr["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBPS,
            "source": "profiles/trace_roofline.json: rocprofv3 --kernel-trace of this command on a committed run "
                      f"({tr.get('run', 'see DESIGN §5')}); the profiler's per-kernel completion handling adds a "
                      "few µs, box-to-box spread ±4 %"}


def _mix_ceiling(mix):
    """The best rate a plain float4 grid reached for the same read / write mix on
    the same number of elements (scripts/micro/stream_mix.hip: no chunk map, no
    descriptors; committed run), as a fraction of 8 TB/s: what this kernel's
    beyond-cache fraction is read against."""
    path = os.path.join(REPO, "profiles", "r4", "r4p_stream_mix_2.jsonl")
    try:
        with open(path) as f:
            rows = [json.loads(ln) for ln in f if ln.strip()]
    except (OSError, ValueError):
        return None
    best = max((r for r in rows if r["case"].startswith(mix)), key=lambda r: r["frac"], default=None)
    if best is None:
        return None
    return {"frac": round(best["frac"], 4), "case": best["case"], "grid": best["grid"],
            "source": "profiles/r4/r4p_stream_mix_2.jsonl (scripts/micro/stream_mix.hip, a plain float4 stream of "
                      "the same mix, ResNet-152 x 2 elements, one MI355X; box-to-box spread a few %)"}


def grad_sync_kernel_rates(params, dev, iters=20, comm=None, world=1):
    """Every grad-sync kernel of the step, after the timed region, warm and alone
    on the GPU, on this model's parameter set (``kernels``) and on a >256 MiB
    working set (``kernels_beyond_ic``: ResNet-152 x 2, true-HBM rates — SURVEY
    §8(d)), against the 8 TB/s HBM peak: the north star's ">= 70 % of HBM peak"
    covers all of them, not just the headline update kernel.  With the engine's
    one-rank RCCL communicator: configs[3]'s N>1 clip path at its N=8 shard."""
    n, rows = _kernel_rows([tuple(p.shape) for p in params], dev, iters)
    n_big, big = _kernel_rows(_beyond_ic_shapes(), dev, iters, shapes16=_beyond_ic_shapes() * 2)
    torch.cuda.empty_cache()
    out = {"params": n, "kernels": rows, "peak_GBps": HBM_PEAK_GBPS, "iters": iters,
           "timing": "after the timed region, warm, alone on the GPU; plan launch timer (the kernels' own start "
                     f"and end: hipExtLaunchKernel's HIP events on the launch stream), average of {iters} calls",
           "min_frac": min(r["frac"] for r in rows.values()),
           "beyond_ic": {"params": n_big, "set": "ResNet-152 parameter shapes x 2 (> 256 MiB Infinity Cache); the "
                                               "16-bit-source rows (pack_bf16, unpack_bf16_to_f32) on x 4: a 481 MB "
                                               "bf16 source",
                         "kernels": big, "min_frac": min(r["frac"] for r in big.values())}}
    if comm is not None and world == 1:
        out.update(zero_clip_path_rows(n, dev, comm, iters=iters))
    live = _live_mix_ceiling(dev)
    out["beyond_ic"]["plain_stream_ceiling_live"] = live
    for name, mix in LIVE_MIX_OF_ROW.items():  # each row against its own mix's plain grid
        if name in big and (live.get(mix) or {}).get("frac"):
            big[name]["frac_of_live_ceiling"] = big[name]["frac"] / live[mix]["frac"]
    return out


# the update rows' mixes as scripts/micro/stream_mix.hip names its plain-stream cases
LIVE_MIX_CASES = {"sgd3r2w": ("sgd3r2w_g2", "sgd3r2w_g4", "sgd3r2w_g4_ntl"),
                  "adam4r3w": ("adam4r3w_g4", "adam4r3w_g4_ntl"),
                  "copy": ("copy_g4", "copy_g4_ntl"), "read": ("read_sum_g4", "read_sum_g4_ntl"),
                  # the 16-bit rows: bf16 -> bf16 (4 B/elem), fp32 -> bf16 and bf16 -> fp32 (6 B/elem)
                  "cvt16_16": ("cvt16_16_e4", "cvt16_16_e8", "cvt16_16_e8_ntl"),
                  "cvt32_16": ("cvt32_16_e4", "cvt32_16_e8", "cvt32_16_e4_ntl"),
                  "cvt16_32": ("cvt16_32_e4", "cvt16_32_e8", "cvt16_32_e8_ntl")}
# the beyond-cache rows whose stream mix one of them is exactly
LIVE_MIX_OF_ROW = {"sgd_momentum_wd": "sgd3r2w", "adam": "adam4r3w", "pack_f32": "copy", "unpack_f32": "copy",
                   "sqnorm_f32": "read", "sqnorm_partial_f32": "read", "pack_bf16": "cvt16_16",
                   "pack_f32_to_bf16": "cvt32_16", "unpack_bf16_to_f32": "cvt16_32"}


def _live_mix_ceiling(dev):
    """The plain-stream ceiling of the update rows' read / write mixes measured on
    THIS box, right after the beyond-cache rows: scripts/micro/stream_mix (built
    in-tree by __graft_entry__.build()) as a child process on the same GPU, the
    mix's one-shot-grid cases on ResNet-152 x 2 elements, each kernel timed by
    its own start / stop events like the plan launch timer; per mix the best case
    (median of 2 rounds x 20 launches).  None (with the reason) when the binary is
    absent or fails."""
    import subprocess

    exe = os.path.join(REPO, "scripts", "micro", "stream_mix")
    if not os.path.exists(exe):
        return {"error": "scripts/micro/stream_mix not built"}
    if (dev.index or 0) != 0:  # the child runs on its default device: the same GPU only for device 0
        return {"error": f"measured on device 0 only (this rank: {dev})"}
    torch.cuda.synchronize(dev)
    cases = [c for cs in LIVE_MIX_CASES.values() for c in cs]
    try:
        p = subprocess.run([exe] + cases, capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.TimeoutExpired) as e:
        return {"error": f"stream_mix: {e!r}"}
    if p.returncode != 0:
        return {"error": f"stream_mix exit {p.returncode}: {p.stderr[-300:]}"}
    rows = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    out = {}
    for mix, names in LIVE_MIX_CASES.items():
        per = {}
        for r in rows:
            if r["case"] in names:
                per.setdefault(r["case"], []).append(r["frac"])
        if per:
            best = max(per, key=lambda c: sorted(per[c])[len(per[c]) // 2])
            fr = sorted(per[best])[len(per[best]) // 2]
            out[mix] = {"frac": round(fr, 4), "GBps": round(fr * HBM_PEAK_GBPS, 1), "case": best,
                        "cases": {c: [round(x, 4) for x in v] for c, v in per.items()}}
    out["source"] = ("scripts/micro/stream_mix.hip run live on this GPU after the beyond-cache rows: a plain float4 "
                     "grid of the same read / write mix on the same 120.4 M elements, no chunk map; kernel start / "
                     "stop events")
    return out


class _BenchColl:
    """The bench's own barriers and MAX-over-ranks: on the engine's libgsync
    communicator when it has one (one RCCL communicator per rank), else on the
    process group."""

    def __init__(self, comm, dev, pg_backend):
        self.comm = comm
        self.dev = dev
        self.pg_backend = pg_backend

    def barrier(self):
        if self.comm is not None:
            t = torch.zeros(1, device=self.dev)
            self.comm.all_reduce(t, stream=torch.cuda.current_stream(self.dev).cuda_stream)
            torch.cuda.synchronize(self.dev)
        else:
            dist.barrier()

    def max(self, x: float) -> float:
        on_dev = self.comm is not None or self.pg_backend == "nccl"
        t = torch.tensor([x], dtype=torch.float64, device=self.dev if on_dev else "cpu")
        if self.comm is not None:
            self.comm.all_reduce(t, op="max", stream=torch.cuda.current_stream(self.dev).cuda_stream)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def _engine_comm(ddp, zero):
    if zero is not None:
        return zero._comm
    for m in (ddp, getattr(ddp, "module", None)):
        c = getattr(m, "_comm", None)
        if c is not None:
            return c
    return None


# Cost estimates of the optional legs after the timed region (seconds), for the
# --wall-budget-s skip decision.  LEG_COST_S is the one-GPU figure: the larger of the
# N=1 runs with every leg on (profiles/r3/r3n_bench_n1_all_legs.json;
# profiles/r5/r5a_bench_legs_n1.json: zero2 1.2 s, colossal 35.3 s) and the 4-rank
# full-size rehearsals divided by their 4 ranks' share of the one GPU
# (profiles/r4/r4d_n4_budget240.json), doubled, at least 5 s; zero2 / colossal include
# their first-step MIOpen compiles; the policy A/B has 8 variants since r5.  leg_cost()
# scales it with the world size:
#   * nccl (one rank per GPU): the ranks' GPU work runs in parallel, so the base holds;
#     what grows with N is each collective's latency and communicator set-up (the A/B's
#     rccl_max_ctas variant and the xgmi calibration bring up / time their own) and the
#     concurrent first-step MIOpen compiles of N processes on the node's host cores:
#     LEG_GROWTH_PER_RANK of the base per extra rank, plus LEG_FIXED_PER_RANK_S for the
#     legs that create communicators;
#   * gloo (the rehearsal: N ranks share the box's GPUs): every rank's GPU work
#     serialises on the shared device — the base times the ranks per GPU — plus the same
#     per-rank growth.
# Both scale with the per-rank batch (the base is 256 images a rank).  Checked against
# the 8-rank rehearsal of the driver's command (gloo, 64 images a rank, round 6,
# profiles/r6/r6n8_n8_gloo.json): zero2 15.8 s against 63 s estimated, the policy A/B
# 23.0 s against 166 s, tail / parity / kernel rates 0.4 / 0.6 / 1.4 s against 5-12 s.
LEG_COST_S = {"tail_split": 5.0, "parity": 5.0, "collective_bench": 10.0, "kernel_rates": 20.0,
              "zero2": 2 * 2 * 18.4 / 4,  # at N > 1 two engines (default + overlap_allgather)
              "colossal": 2 * 63.6 / 2, "bucket_policy_ab": 2 * 35.0 * 8 / 6 / 2, "torch_ddp": 10.0,
              "torch_colossal": 30.0}
LEG_GROWTH_PER_RANK = 0.10
# torch's own DDP over gloo stages every bucket through the host per rank: its legs ran
# 3.7x / 2.6x their estimates in the 8-rank rehearsal (profiles/r6/r6n8c_n8_gloo.json)
LEG_GLOO_FACTOR = {"torch_ddp": 4.0, "torch_colossal": 3.0}
LEG_FIXED_PER_RANK_S = {"bucket_policy_ab": 1.0, "zero2": 0.25, "colossal": 0.25, "collective_bench": 0.25}


def leg_cost(name, world, backend, ranks_per_gpu=1, batch=256):
    """Estimated seconds of leg `name` at `world` ranks of `batch` images (see LEG_COST_S)."""
    base = LEG_COST_S.get(name, 5.0)
    if backend == "gloo":
        base *= LEG_GLOO_FACTOR.get(name, 1.0)
    share = (max(1, ranks_per_gpu) if backend == "gloo" else 1) * max(batch, 1) / 256.0
    return max(5.0, base * share * (1.0 + LEG_GROWTH_PER_RANK * (world - 1))
               + LEG_FIXED_PER_RANK_S.get(name, 0.0) * (world - 1))


# the reference's DeepSpeed optimizer (R:resnet/deepspeed/deepspeed_train.py:175-186): "Adam" in
# AdamW mode, betas (0.8, 0.999), eps 1e-8, weight_decay 3e-7; gradient_clipping 1.0 (:195)
DS_ADAM = dict(lr=1e-3, betas=(0.8, 0.999), eps=1e-8, weight_decay=3e-7)


# DESIGN §8 decision rule for the bucket policy (row N1), fixed before the
# driver's N > 1 run: a variant replaces the torch layout as the default when
# its images/s beat the mean of the two torch-layout runs (before and after,
# to cancel drift) by >= 0.5 % with parity.ok; the best such variant wins.
POLICY_MARGIN = 0.005


def bucket_policy_ab(model, opt, ddp, x, y, crit, world, dev, args, steps=8):
    """Re-wrap `model` with each bucket policy and time `steps` steps of each
    (after a one-bucket first step and the rebuild step), rank-synchronised
    and MAX over ranks like the headline; per variant: images/s, the exposed
    tail (timed steps) and its split, in-step and standalone all-reduce bus
    bandwidth against (n-1) x 153 GB/s, and the self-checked parity step."""
    import distributed_training_amd as D
    from distributed_training_amd import parity as PC

    bucket_dtype = torch.bfloat16 if args.bucket_dtype == "bf16" else None
    # bf16_buckets: half the bytes on the links, but other numerics (opt-in) — reported,
    # never a candidate for the default
    # gradient_as_bucket_view (no unpack: the grads are bucket views) and the overlapped
    # optimizer (each bucket's update behind its unpack, under backward) shorten the
    # exposed tail with the numerics unchanged: candidates like the layouts
    variants = [("torch", {}), ("xgmi", {"bucket_policy": "xgmi"}),
                ("last_bucket_cap_1MiB", {"last_bucket_cap_mb": 1.0}),
                *([("bf16_buckets", {"bucket_dtype": torch.bfloat16})] if bucket_dtype is None else []),
                ("rccl_cta_cap_16", {"rccl_max_ctas": 16}),
                ("grad_as_bucket_view", {"gradient_as_bucket_view": True}),
                ("optimizer_overlap", {"optimizer_overlap": True}),
                ("torch_again", {})]
    ddp.close()
    peak = (world - 1) * XGMI_LINK_GBPS
    rows = {}
    for name, kw in variants:
        kw = dict(kw)
        bdt = kw.pop("bucket_dtype", bucket_dtype)
        gview = kw.pop("gradient_as_bucket_view", args.grad_as_bucket_view)
        overlap = kw.pop("optimizer_overlap", False)
        try:
            v = D.DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb, bucket_dtype=bdt,
                                          gradient_as_bucket_view=gview, **kw)
        except Exception as e:  # e.g. RCCL refusing a communicator config: every rank alike
            rows[name] = {"error": f"{type(e).__name__}: {e}"[:300], "parity": None}
            continue
        vopt = opt
        if overlap:
            if args.optimizer == "sgd":
                v._register_fused_optim(torch.optim.SGD, lr=0.1, momentum=0.9, weight_decay=1e-4)
            else:
                v._register_fused_optim(torch.optim.Adam, lr=1e-3 * world)
            vopt = _OverlappedStep(v)

        def fwd_bwd():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = crit(v(x), y)
            loss.backward()

        def one():
            fwd_bwd()
            vopt.step()
            vopt.zero_grad(set_to_none=True)

        for _ in range(2):
            one()
        torch.cuda.synchronize()
        c = _BenchColl(v._comm, dev, args.pg_backend)
        c.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
        c.barrier()
        el = c.max(time.perf_counter() - t0)
        tail_timed = v.tail_ms()
        v.set_timeline(2)
        one()
        torch.cuda.synchronize()
        comm_ms = [m for m in v.bucket_comm_ms() if m >= 0]
        tail = v.tail_ms()
        v.set_timeline(1)
        bucket_bytes = [b.numel() * b.element_size() for b in v._bucketer.buffers]
        row = {"images_per_sec": world * args.batch * steps / el, "ms_per_step": el / steps * 1e3,
               "bucket_bytes": bucket_bytes, "tail_ms_timed": tail_timed["total"] if tail_timed else None,
               "tail_split_ms": tail}
        if world > 1 and comm_ms and min(comm_ms) > 0:
            bus = sum(bucket_bytes) / (sum(comm_ms) * 1e-3) * 2 * (world - 1) / world / 1e9
            row["in_step_bus_GBps"] = bus
            row["in_step_frac"] = bus / peak
        if v._comm is not None and world > 1:
            sa = collective_bench(v, None, world)
            row["standalone"] = {"bus_GBps": sa["bus_GBps"], "frac": sa["frac"], "ms_per_step": sa["ms_per_step"],
                                 "whole_grad": next((r for r in sa["per_op"] if r["op"] == "all_reduce_whole_grad"),
                                                    None)}
        cal = v._get_ddp_logging_data().get("xgmi_calibration")
        if cal:
            row["xgmi_calibration"] = cal
        row["parity"] = PC.ddp_parity_step(v, vopt, fwd_bwd)
        rows[name] = row
        v.close()
    base = (rows["torch"]["images_per_sec"] + rows["torch_again"]["images_per_sec"]) / 2
    best, best_ips = "torch", base * (1 + POLICY_MARGIN)
    if "images_per_sec" in rows.get("bf16_buckets", {}):
        rows["bf16_buckets"]["vs_torch"] = rows["bf16_buckets"]["images_per_sec"] / base
    for name in ("xgmi", "last_bucket_cap_1MiB", "rccl_cta_cap_16", "grad_as_bucket_view", "optimizer_overlap"):
        r = rows[name]
        if "error" in r:
            continue
        r["vs_torch"] = r["images_per_sec"] / base
        if r["parity"] and r["parity"].get("ok") and r["images_per_sec"] >= best_ips:
            best, best_ips = name, r["images_per_sec"]
    return {"variants": rows, "steps_each": steps, "torch_mean_images_per_sec": base,
            "rule": f"a variant becomes the default if images/s >= (1 + {POLICY_MARGIN}) x the mean of the two "
                    "torch-layout runs with parity.ok (DESIGN §8); best such variant wins; bf16_buckets is "
                    "reported only (other numerics)",
            "decision": best}


def _zero2_run(args, world, rank, dev, coll_h, steps, warmup, overlap_allgather=False):
    """One configs[3] engine on a fresh bf16 ResNet-50: `steps` timed steps (MAX
    over ranks), the shard update's launches, the end-of-step all-gather timed on
    one more step (HIP events around it on the step's stream: its exposed time),
    and the self-checked parity step."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd import parity as PC
    from distributed_training_amd.resnet import MODELS
    from distributed_training_amd.zero import ZeroDataParallel

    torch.manual_seed(0)
    model = MODELS[args.model](num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    zero = ZeroDataParallel(model, stage=2, optimizer="adamw", momentum=0.9, reduce_bucket_size=int(5e7),
                            gradient_clipping=1.0, overlap_allgather=overlap_allgather, **DS_ADAM)
    g = torch.Generator(device=dev).manual_seed(4321 + rank)
    x = torch.rand(args.batch, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    x = x.to(torch.bfloat16)
    y = torch.randint(0, 1000, (args.batch,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    def fwd_bwd():
        crit(model(x).float(), y).backward()

    def one():
        zero.prepare_backward()
        fwd_bwd()
        zero.step()

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    zero.plan.timer_enable(4 * steps + 8)
    coll_h.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    coll_h.barrier()
    el = coll_h.max(time.perf_counter() - t0)
    upd = zero.plan.timer_read(kind=L.GS_OP_ADAM)
    zero.plan.timer_enable(0)
    zero.time_allgather(True)
    one()
    ag_ms = zero.last_allgather_ms()
    zero.time_allgather(False)
    shard = sum(zero.shard_sizes)
    upd_ms = sum(upd) / len(upd) if upd else None
    out = {"images_per_sec": world * args.batch * steps / el, "ms_per_step": el / steps * 1e3,
           "per_gpu_batch": args.batch, "steps": steps, "warmup": warmup, "buckets": len(zero.buckets),
           "shard_update": {"avg_launch_ms": upd_ms, "alg_bytes_per_launch": 28 * shard,
                            "frac": 28 * shard / (upd_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS if upd_ms else None},
           "allgather_exposed_ms": ag_ms,
           "allgather_timing": ("HIP events around the end-of-step all-gathers on the step's stream, one step "
                                "after the timed region" + ("; overlap_allgather: their issue only, the gathers "
                                                            "run on the communicator's stream under the next "
                                                            "forward" if overlap_allgather else ""))}
    zero.wait_allgather()
    # the step's end (update + its collectives): HIP events right around zero.step() on
    # the step's stream, median of 6 untimed steps each, with the collectives' watchdog
    # marks on the consuming kernels (the default) and with round 5's event packet after
    # every collective — the same run, the same GPU
    def step_end_ms(packets):
        zero.set_mark_packets(packets)
        evs = []
        for _ in range(6):
            zero.prepare_backward()
            fwd_bwd()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            zero.step()
            b.record()
            evs.append((a, b))
        torch.cuda.synchronize()
        zero.set_mark_packets(False)
        return sorted(x.elapsed_time(y) for x, y in evs)[len(evs) // 2]

    if zero._comm is not None and zero._comm.timeout_ms > 0:
        marked, packets = step_end_ms(False), step_end_ms(True)
        out["step_end_window"] = {
            "ms": marked, "ms_with_packets_r5": packets, "saved_us": (packets - marked) * 1e3,
            "timing": "HIP events around zero.step() on the step's stream (median of 6 untimed steps): the update, "
                      "the clip / overflow all-reduces and the parameter all-gathers; 'with_packets_r5': an event "
                      "packet after every collective for the RCCL watchdog, as round 5"}
    zero.wait_allgather()
    out["parity"] = PC.zero_parity_step(zero, fwd_bwd)
    zero.close()
    del zero, model
    torch.cuda.empty_cache()
    return out


def zero2_leg(args, world, rank, dev, coll_h, steps=8, warmup=3):
    """BASELINE configs[3] on the same ranks as the headline: a fresh ResNet-50
    in bf16 on the libgsync ZeRO-2 engine as the DeepSpeed config drives it
    (R:resnet/deepspeed/deepspeed_train.py:170-219: bf16, stage 2, AdamW,
    gradient_clipping 1.0, reduce_bucket_size 5e7; reduce-scatter of bf16
    grads, fp32 master shard update, all-gather of bf16 params) on the same
    communicator, `steps` timed steps (MAX over ranks) and one self-checked
    step.  At N > 1 also the opt-in overlapped all-gather (ZeroDataParallel
    overlap_allgather: per-bucket gathers under the next forward), timed and
    parity-checked the same way."""
    out = {"engine": "zero2", "config": "BASELINE configs[3]: ResNet-50 bf16 model, ZeRO-2 reduce-scatter + "
                                        "AdamW on fp32 master shards + all-gather, clip 1.0",
           "optimizer": dict(DS_ADAM, kind="adamw", gradient_clipping=1.0)}
    out.update(_zero2_run(args, world, rank, dev, coll_h, steps, warmup))
    if world > 1:
        out["overlap_allgather"] = _zero2_run(args, world, rank, dev, coll_h, steps, warmup, overlap_allgather=True)
    return out


def colossal_leg(args, world, rank, dev, coll_h, batch=128, steps=8, warmup=8):
    """BASELINE configs[4] inside the N > 1 run: a fresh ResNet-152 (fp32
    params and grads, 240.8 MB all-reduced a step) through the Colossal shim as
    R:resnet/colossal/run.sh drives it (TorchDDPPlugin, mixed_precision='fp16',
    HybridAdam(lr=1e-3*ws), R:resnet/colossal/colossal_train.py:118-161):
    libgsync DDP underneath, GradScaler's inf check fused into the unpack.
    `steps` timed steps (MAX over ranks) and one self-checked step; the warm-up
    lets the fp16 loss scale settle (from 2**16 it backs off on the first
    steps' overflows, whose update launches exit at once and are not timed)."""
    import distributed_training_amd as D
    from distributed_training_amd import parity as PC
    from distributed_training_amd.compat import colossalai as C
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    name = "resnet152" if args.model == "resnet50" else args.model  # small rehearsals keep their small model
    model = MODELS[name](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    booster = C.Booster(plugin=C.TorchDDPPlugin(), mixed_precision="fp16")
    opt = C.HybridAdam(model.parameters(), lr=1e-3 * world)
    cmodel, opt_w, ccrit, _, _ = booster.boost(model, opt, criterion=torch.nn.CrossEntropyLoss())
    ddp = next(m for m in cmodel.modules() if isinstance(m, D.DistributedDataParallel))
    g = torch.Generator(device=dev).manual_seed(5678 + rank)
    x = torch.rand(batch, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev, generator=g)

    def fwd_bwd():
        booster.backward(ccrit(cmodel(x), y), opt_w)

    def one():
        fwd_bwd()
        opt_w.step()
        opt_w.zero_grad()

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    opt.enable_kernel_timer(steps + 4)  # HybridAdam = libgsync FusedAdam: its update launches
    flags = []
    coll_h.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
        flags.append(opt_w.scaler._state(opt_w.optim)["found_inf"].clone())  # device copy, no sync
    torch.cuda.synchronize()
    coll_h.barrier()
    el = coll_h.max(time.perf_counter() - t0)
    n_params = sum(p.numel() for p in ddp._params)
    # fp16 GradScaler: an overflowing step's update exits at once on the device flag;
    # only the launches that updated count toward the rate (as the colossal engine's headline)
    ms = opt.kernel_ms()
    upd = [m for m, f in zip(ms, flags) if f.item() == 0] if len(ms) == len(flags) else ms
    opt.enable_kernel_timer(0)
    upd_ms = sum(upd) / len(upd) if upd else None
    out = {"engine": "colossal", "model": name,
           "config": "BASELINE configs[4]: ResNet-152 fp32 params/grads through the Colossal "
                     "Booster(TorchDDPPlugin, fp16) + HybridAdam, libgsync DDP underneath",
           "images_per_sec": world * batch * steps / el, "ms_per_step": el / steps * 1e3, "per_gpu_batch": batch,
           "steps": steps, "warmup": warmup, "grad_bytes_per_step": 4 * n_params,
           "fused_adam": {"avg_launch_ms": upd_ms, "alg_bytes_per_launch": 28 * n_params,
                          "frac": 28 * n_params / (upd_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS if upd_ms else None,
                          "launches": len(upd), "skipped_launches": len(ms) - len(upd),
                          "timing": "libgsync plan launch timer (the kernel's own start / end), the timed steps"}}
    out["parity"] = PC.ddp_parity_step(ddp, opt_w, fwd_bwd)
    opt_w.zero_grad()
    ddp.close()
    del cmodel, opt_w, ddp, model
    torch.cuda.empty_cache()
    return out


def _time_torch_steps(one, world, batch, dev, steps, warmup):
    """`warmup` untimed steps, then `steps` timed ones bracketed by barrier +
    synchronize on both sides, MAX over ranks (the headline's bracket)."""
    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    # per-step durations of a few more steps (events on the current stream): a warm-up
    # that did not settle shows as a trend here
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
    for a, b in evs:
        a.record()
        one()
        b.record()
    torch.cuda.synchronize()
    return {"images_per_sec": world * batch * steps / el, "ms_per_step": el / steps * 1e3, "steps": steps,
            "after_ms": [round(a.elapsed_time(b), 3) for a, b in evs],
            "warmup": warmup, "per_gpu_batch": batch,
            "timing": "barrier + synchronize on both sides, MAX over ranks (as the headline)"}


def torch_ddp_leg(args, world, rank, dev, mf, steps=20, warmup=3):
    """The reference's own GPU path beside the headline, in the same run (VERDICT r5
    next 5): a fresh model of the same architecture and seed, torch's
    DistributedDataParallel over the nccl (RCCL) process group, bf16 autocast,
    torch.optim.SGD(lr 0.1, momentum 0.9, wd 1e-4, foreach) — the headline's step with
    torch's Reducer and foreach optimizer in place of libgsync
    (R:resnet/pytorch_ddp/ddp_train.py:95-97 wraps the model in DDP and steps a
    torch.optim optimizer) — `steps` timed steps bracketed like the headline's."""
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    model = MODELS[args.model](num_classes=1000).to(dev).to(memory_format=mf)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index], bucket_cap_mb=args.bucket_cap_mb)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(args.batch, 3, 224, 224, device=dev, generator=g).to(memory_format=mf)
    y = torch.randint(0, 1000, (args.batch,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    def one():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    out = dict(impl="torch DistributedDataParallel + torch.optim.SGD(foreach), bf16 autocast, channels_last",
               **_time_torch_steps(one, world, args.batch, dev, steps, warmup))
    del ddp, opt, model
    torch.cuda.empty_cache()
    return out


def torch_colossal_leg(args, world, rank, dev, batch=128, steps=8, warmup=10):
    """configs[4] on torch alone beside the colossal leg, same run: what
    TorchDDPPlugin + mixed_precision='fp16' + HybridAdam run as on torch
    (R:resnet/colossal/colossal_train.py:118-161): torch DDP, fp16 autocast with
    the criterion inside, torch.amp.GradScaler, torch.optim.AdamW(fused, lr
    1e-3 x ws, weight_decay 0), ResNet-152 at the colossal leg's batch."""
    from distributed_training_amd.resnet import MODELS

    name = "resnet152" if args.model == "resnet50" else args.model
    torch.manual_seed(0)
    model = MODELS[name](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3 * world, weight_decay=0.0, fused=True)
    scaler = torch.amp.GradScaler("cuda")
    g = torch.Generator(device=dev).manual_seed(5678 + rank)
    x = torch.rand(batch, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    def one():
        with torch.autocast("cuda", dtype=torch.float16):
            loss = crit(ddp(x), y)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        opt.zero_grad(set_to_none=True)

    out = dict(impl="torch DDP + fp16 autocast + torch.amp.GradScaler + torch.optim.AdamW(fused)", model=name,
               **_time_torch_steps(one, world, batch, dev, steps, warmup))
    del ddp, opt, model
    torch.cuda.empty_cache()
    return out


class _OverlappedStep:
    """The bench's optimizer handle under --optimizer-overlap: the update already
    ran per bucket inside backward, so step() is empty; kernel_ms() is the sum
    over the buckets' launches of each step (one whole-model update per step)."""

    def __init__(self, ddp):
        self.ddp = ddp
        self.main = ddp._overlapped_optimizer

    def _opts(self):
        return [o for o in self.ddp._overlap["per_bucket"].values() if o]

    def step(self):
        pass

    def zero_grad(self, set_to_none=True):
        self.main.zero_grad(set_to_none=set_to_none)

    def enable_kernel_timer(self, n):
        for o in self._opts():
            o.enable_kernel_timer(n)

    def kernel_ms(self):
        per = [o.kernel_ms() for o in self._opts()]
        n = min((len(x) for x in per), default=0)
        return [sum(x[k] for x in per) for k in range(n)]


def main():
    args = parse()
    if os.environ.get("GSYNC_BENCH_TRACEBACK_S"):  # debugging aid: every rank's stacks every N s
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["GSYNC_BENCH_TRACEBACK_S"]), repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    init_method = None  # env:// (torch.distributed.run's store) at N > 1
    if world == 1:
        # one rank: a file store — no TCP port to race for (a port picked free can be
        # taken by another process's ephemeral socket before the store listens on it)
        import tempfile

        store_path = os.path.join(tempfile.gettempdir(), f"gsync_bench_{os.getpid()}_{time.time_ns()}")
        init_method = "file://" + store_path
        import atexit

        atexit.register(lambda: os.path.exists(store_path) and os.remove(store_path))
    if args.pg_backend == "gloo":
        # rehearsal of the N > 1 control flow on a box with fewer GPUs than ranks:
        # ranks share the devices round-robin and the bucket collectives go through
        # gloo (RCCL refuses two ranks on one GPU); never the measured configuration
        dev = torch.device("cuda", local_rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method=init_method)
    else:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        # libgsync brings up its own RCCL communicator (unique id through the store) and
        # the bench's barriers / MAX go through it (_BenchColl): no device_id, so torch's
        # ProcessGroupNCCL never builds a second communicator on the rank; --impl torch
        # uses the process group itself (eager init)
        kw = dict(device_id=dev) if args.impl == "torch" else {}
        dist.init_process_group("nccl", rank=rank, world_size=world, init_method=init_method, **kw)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)

    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS

    classes = 1000
    torch.manual_seed(0)
    model = MODELS[args.model](num_classes=classes).to(dev)
    mf = torch.contiguous_format if args.no_channels_last else torch.channels_last
    model = model.to(memory_format=mf)
    bucket_dtype = torch.bfloat16 if args.bucket_dtype == "bf16" else None
    n_params = sum(p.numel() for p in model.parameters())
    zero = None
    torch_zero = args.impl == "torch" and args.engine == "zero2"
    if torch_zero:
        # configs[3] on torch alone: FSDP SHARD_GRAD_OP is ZeRO-2 (grads reduce-scattered, params
        # replicated); bf16 compute / reduce-scatter over fp32 master shards as DeepSpeed's bf16
        # mode; fused AdamW, clip 1.0 (R:resnet/deepspeed/deepspeed_train.py:170-219)
        if args.graph:
            raise SystemExit("--impl torch: eager only")
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP, MixedPrecision, ShardingStrategy

        bf = torch.bfloat16
        ddp = FSDP(model, sharding_strategy=ShardingStrategy.SHARD_GRAD_OP, device_id=dev,
                   mixed_precision=MixedPrecision(param_dtype=bf, reduce_dtype=bf, buffer_dtype=bf))
        opt = torch.optim.AdamW(ddp.parameters(), fused=True, **DS_ADAM)
        bytes_per_param = 28
        grad_bytes = n_params * 2
    elif args.impl == "torch":
        if args.engine not in ("ddp", "colossal") or args.graph:
            raise SystemExit("--impl torch: DDP, colossal or zero2 engine, eager only")
        ddp = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[dev.index] if args.pg_backend == "nccl" else None,
            bucket_cap_mb=args.bucket_cap_mb, gradient_as_bucket_view=args.grad_as_bucket_view)
        if args.engine == "colossal":
            # what Colossal's TorchDDPPlugin + mixed_precision='fp16' + HybridAdam run on torch alone:
            # torch DDP, fp16 autocast (criterion inside), torch.amp.GradScaler, fused AdamW
            # (HybridAdam(adamw_mode=True), weight_decay 0: R:resnet/colossal/colossal_train.py:118-161)
            opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3 * world, weight_decay=0.0, fused=True)
            torch_scaler = torch.amp.GradScaler("cuda")
            bytes_per_param = 28
        elif args.optimizer == "sgd":
            opt = torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
            bytes_per_param = 20
        else:
            opt = torch.optim.Adam(ddp.parameters(), lr=1e-3 * world, foreach=True)
            bytes_per_param = 28
        grad_bytes = n_params * 4
    elif args.engine == "ddp":
        ddp = D.DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb, bucket_dtype=bucket_dtype,
                                        gradient_as_bucket_view=args.grad_as_bucket_view,
                                        bucket_policy=args.bucket_policy, last_bucket_cap_mb=args.last_bucket_cap_mb)
        if args.optimizer_overlap:
            if args.graph:
                raise SystemExit("--optimizer-overlap: eager only")
            if args.optimizer == "sgd":
                ddp._register_fused_optim(torch.optim.SGD, lr=0.1, momentum=0.9, weight_decay=1e-4)
            else:
                ddp._register_fused_optim(torch.optim.Adam, lr=1e-3 * world)
            opt = _OverlappedStep(ddp)
            bytes_per_param = 20 if args.optimizer == "sgd" else 28
        elif args.optimizer == "sgd":
            opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4,
                             capturable=bool(args.graph))
            bytes_per_param = 20  # p r/w, g r, buf r/w (fp32)
        else:
            opt = D.FusedAdam(ddp.parameters(), lr=1e-3 * world, capturable=bool(args.graph))
            bytes_per_param = 28
        grad_bytes = n_params * (2 if bucket_dtype is not None else 4)
    elif args.engine == "colossal":
        # BASELINE configs[4] through the Colossal shim exactly as R:resnet/colossal/run.sh drives it:
        # TorchDDPPlugin + mixed_precision='fp16' + HybridAdam(lr=1e-3*ws) (R:colossal_train.py:118-161);
        # fp32 params and grads, libgsync DDP underneath, GradScaler's check fused into the unpack
        from distributed_training_amd.compat import colossalai as C

        booster = C.Booster(plugin=C.TorchDDPPlugin(), mixed_precision="fp16")
        opt = C.HybridAdam(model.parameters(), lr=1e-3 * world)
        cmodel, opt_w, ccrit, _, _ = booster.boost(model, opt, criterion=torch.nn.CrossEntropyLoss())
        ddp = cmodel.module  # _AutocastModule(libgsync DDP)
        bytes_per_param = 28
        grad_bytes = n_params * 4
    else:
        # DeepSpeed-style ZeRO (BASELINE configs[3]): bf16 model, fp32 master shard,
        # reduce-scatter (zero2) / all-reduce (zero1) of bf16 grads, AdamW, all-gather
        from distributed_training_amd.zero import ZeroDataParallel

        model = model.to(torch.bfloat16)
        zero = ZeroDataParallel(model, stage=2 if args.engine == "zero2" else 1,
                                optimizer="sgd" if args.optimizer == "sgd" else "adamw",
                                momentum=0.9, reduce_bucket_size=int(5e7), gradient_clipping=1.0, **DS_ADAM)
        ddp = model
        # per shard param: p r/w fp32, g r bf16, states r/w fp32, bf16 param write
        bytes_per_param = (4 + 4 + 2 + 8 + 2) if args.optimizer == "sgd" else (4 + 4 + 2 + 16 + 2)
        grad_bytes = n_params * 2

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(args.batch, 3, 224, 224, device=dev, generator=g).to(memory_format=mf)
    y = torch.randint(0, classes, (args.batch,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    ev_opt = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    if zero is not None or torch_zero:
        x = x.to(torch.bfloat16)

    def step(i=None):
        if zero is not None:
            zero.prepare_backward()
            loss = crit(ddp(x).float(), y)
            loss.backward()
            if i is not None:
                ev_opt[i][0].record()
            zero.step()
            if i is not None:
                ev_opt[i][1].record()
            return loss
        return run(x, y)

    def train_step(xb, yb):
        if args.graph:
            # released before every eager warm-up step and before the recording: the
            # recorded backward then writes fresh grads in the graph's pool, reused by
            # every replay (set_to_none=False would record a zero fill + an accumulate
            # per parameter: ~1 ms a step at ResNet-50, profiles/r2graph/)
            opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = ddp(xb)
            loss = crit(out, yb)
        loss.backward()
        opt.step()
        if not args.graph:
            opt.zero_grad(set_to_none=True)
        return loss

    skip_flags = []  # colossal engine: per-step GradScaler found-inf flags (device copies, no sync)

    def colossal_step(xb, yb):  # R:resnet/colossal/colossal_train.py:97-102
        loss = ccrit(cmodel(xb), yb)
        booster.backward(loss, opt_w)
        opt_w.step()
        if record_skips[0]:
            skip_flags.append(opt_w.scaler._state(opt_w.optim)["found_inf"].clone())
        opt_w.zero_grad()
        return loss

    record_skips = [False]

    def torch_colossal_step(xb, yb):  # the same step on torch's own DDP / GradScaler / fused AdamW
        with torch.autocast("cuda", dtype=torch.float16):
            loss = crit(ddp(xb), yb)
        torch_scaler.scale(loss).backward()
        torch_scaler.step(opt)
        torch_scaler.update()
        opt.zero_grad(set_to_none=True)
        return loss

    def torch_zero_step(xb, yb):  # FSDP(SHARD_GRAD_OP) step: bf16 forward/backward, clip, fused AdamW
        loss = crit(ddp(xb).float(), yb)
        loss.backward()
        ddp.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    run = (torch_colossal_step if args.impl == "torch" else colossal_step) if args.engine == "colossal" else \
        torch_zero_step if torch_zero else train_step
    if args.graph:
        if zero is not None:
            raise SystemExit("--graph: DDP engine only")
        run = D.CapturedStep(train_step, optimizers=[opt], warmup=max(1, args.warmup - 1))

    t_w0 = time.time()
    for i in range(args.warmup):
        t_i = time.time()
        step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup step {i}: {time.time() - t_i:.2f}s", file=sys.stderr, flush=True)
    warm_s = time.time() - t_w0

    comm_ms = []
    if args.impl == "torch":
        pass
    elif zero is None:
        opt.enable_kernel_timer(args.steps + 4)
    else:
        zero.plan.timer_enable(4 * args.steps + 8)  # + the Σg² launches of the clip
    record_skips[0] = args.engine == "colossal" and args.impl == "libgsync"
    coll_h = _BenchColl(_engine_comm(ddp, zero) if args.impl == "libgsync" else None, dev, args.pg_backend)
    coll_h.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    record_skips[0] = False
    torch.cuda.synchronize()
    coll_h.barrier()
    elapsed = coll_h.max(time.perf_counter() - t0)
    # the timed launches' kernel durations, read before any untimed step below adds more
    opt_ms_saved = zero_ms_saved = None
    if args.impl == "libgsync" and not args.graph:
        if zero is None:
            opt_ms_saved = opt.kernel_ms()
        else:
            from distributed_training_amd import _lib as L

            zero_ms_saved = zero.plan.timer_read(kind=L.GS_OP_SGD if args.optimizer == "sgd" else L.GS_OP_ADAM)
    # the headline's own numbers, complete before any leg below
    if args.impl == "torch":
        opt_ms = []
    elif zero is None and args.graph:
        # replays carry no timing events: time the update kernel over a few eager
        # launches on the same state after the timed region (same kernel, same plan)
        opt.enable_kernel_timer(8)
        for _ in range(5):
            opt.step()
        torch.cuda.synchronize()
        opt_ms = sorted(opt.kernel_ms())
    elif zero is None:
        # update-kernel launches, HIP events recorded by libgsync on the launch stream
        # right around each kernel (the pointer-table upload, if any, stays outside)
        opt_ms = opt_ms_saved
        if skip_flags and len(skip_flags) == len(opt_ms):
            # fp16 GradScaler: an overflowing step's update kernel exits at once on the
            # device flag; only the launches that updated count toward the rate
            skipped = [f.item() != 0 for f in skip_flags]
            opt_ms = [ms for ms, sk in zip(opt_ms, skipped) if not sk]
        opt_ms = sorted(opt_ms)
    else:
        # the fused shard update alone (plan launch timer); the whole zero.step() window
        # (norm, clip, update, all-gather) is reported beside it
        opt_ms = sorted(zero_ms_saved)
        win_ms = sorted(a.elapsed_time(b) for a, b in ev_opt)
    opt_ms_avg = sum(opt_ms) / len(opt_ms) if opt_ms else None
    img_s = world * args.batch * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3

    upd_params = n_params if zero is None else n_params // world  # ZeRO updates this rank's shard
    achieved = bytes_per_param * upd_params / (opt_ms_avg * 1e-3) / 1e9 if opt_ms_avg else None
    traffic = None
    if os.path.exists(args.traffic_json) and zero is None:
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            key = f"{args.model}/{args.optimizer}"
            traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # the same launches' kernel durations from the committed rocprofv3 kernel trace of
    # this command (scripts/trace_bench.py)
    trace_check = None
    if (zero is None and args.impl == "libgsync" and args.engine == "ddp" and args.model == "resnet50"
            and not args.graph):
        trace_check = _trace_check("SgdOp" if args.optimizer == "sgd" else "AdamOp", bytes_per_param * upd_params)
    if torch_zero:
        log = {"has_rebuilt_buckets": 0}
        bucket_bytes = []
    elif args.impl == "torch":
        log = ddp._get_ddp_logging_data()
        bucket_bytes = [int(b) for b in str(log.get("rebuilt_bucket_sizes", "")).split(",") if b.strip()]
    elif zero is None:
        log = ddp._get_ddp_logging_data()
        bucket_bytes = [b.numel() * b.element_size() for b in ddp._bucketer.buffers]
    else:
        log = {"has_rebuilt_buckets": 0}
        bucket_bytes = [b.numel() * b.element_size() for b in zero.grad_bufs]

    def _roofline():
        kernel = ("gs fused Adam update (chunk_kernel<AdamOp>, HybridAdam via the Colossal shim)"
                  if args.engine == "colossal" else
                  f"gs fused {'SGD' if args.optimizer == 'sgd' else 'Adam'} update "
                  f"(chunk_kernel<{'SgdOp' if args.optimizer == 'sgd' else 'AdamOp'}>)"
                  if zero is None else
                  f"gs ZeRO shard update (chunk_kernel<{'SgdOp' if args.optimizer == 'sgd' else 'AdamOp'}> "
                  f"+ bf16 param write)")
        in_step = {
            "achieved": achieved,
            "frac": achieved / HBM_PEAK_GBPS if achieved else None,
            "frac_of_copy_ceiling": achieved / HBM_COPY_GBPS if achieved else None,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_per_param * upd_params,
            "avg_launch_ms": opt_ms_avg,
            "median_launch_ms": opt_ms[len(opt_ms) // 2] if opt_ms else None,
            "launches": len(opt_ms),
            "timing": ("libgsync plan launch timer: the kernel's own start / end, hipExtLaunchKernel's HIP events "
                       "on the launch stream, the timed steps' launches"
                       + ("; graph mode: 5 eager launches after the timed region" if args.graph else "")
                       + ("; optimizer overlap: per step, the sum of the per-bucket launches (under backward)"
                          if args.optimizer_overlap else "")),
            **({"skipped_launches": sum(f.item() != 0 for f in skip_flags)} if skip_flags else {}),
            **({"rocprof": trace_check} if trace_check else {}),
        }
        # reads above the copy ceiling come partly from the 256 MiB Infinity Cache
        in_step["ic_assisted"] = bool(achieved and achieved > HBM_COPY_GBPS)
        bic = _beyond_ic_roofline(kernel_rates, zero, args, args.traffic_json)
        head = bic if bic else in_step
        r = {"kernel": kernel, "bound": "hbm", "achieved": head["achieved"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
             "frac": head["frac"], "traffic": head["traffic"],
             "algorithmic_bytes_per_launch": head["algorithmic_bytes_per_launch"],
             "avg_launch_ms": head["avg_launch_ms"], "launches": head["launches"],
             "copy_ceiling": HBM_COPY_GBPS,
             "frac_of_copy_ceiling": head["achieved"] / HBM_COPY_GBPS if head["achieved"] else None,
             "working_set": (f"beyond the Infinity Cache: {bic['set']}, {bic['algorithmic_bytes_per_launch'] / 1e9:.2f} "
                             "GB per launch (true HBM)") if bic else
                            f"in the training step ({args.model}; ic_assisted = {in_step['ic_assisted']})",
             "timing": head["timing"]}
        if bic:
            r["frac_beyond_ic"] = bic["frac"]
            r["plain_stream_ceiling"] = bic["plain_stream_ceiling"]
            live = (kernel_rates or {}).get("beyond_ic", {}).get("plain_stream_ceiling_live") or {}
            mix = live.get("sgd3r2w" if args.optimizer == "sgd" else "adam4r3w")
            if mix:
                r["plain_stream_ceiling_live"] = dict(mix, source=live.get("source"))
                r["frac_of_live_ceiling"] = bic["frac"] / mix["frac"] if mix["frac"] else None
            elif live.get("error"):
                r["plain_stream_ceiling_live"] = {"error": live["error"]}
            if "rocprof" in bic:
                r["rocprof"] = bic["rocprof"]
            r["in_step"] = in_step
        else:
            r.update({k: v for k, v in in_step.items() if k not in r})
        return r

    def make_line():
        grad_sync = {"bucket_bytes": bucket_bytes, "n_buckets": len(bucket_bytes), "grad_bytes_per_step": grad_bytes}
        if comm_ms:
            grad_sync["in_step_collective_ms"] = comm_ms
        if world > 1 and comm_ms and min(comm_ms) > 0:
            tot_ms = sum(comm_ms)
            bus = sum(bucket_bytes) / (tot_ms * 1e-3) * 2 * (world - 1) / world / 1e9
            peak = (world - 1) * XGMI_LINK_GBPS
            grad_sync.update({"allreduce_ms_per_step": tot_ms, "allreduce_bus_GBps": bus, "xgmi_peak_GBps": peak,
                              "frac": bus / peak, "per_bucket_ms": comm_ms,
                              "note": "in-step: HIP events around each bucket collective on the comm stream, "
                                      "an untimed step after the timed region (timeline level 2), includes "
                                      "cross-rank arrival skew under backward"})
        if coll is not None:
            grad_sync["standalone"] = coll
        if tail is not None:
            # total: the last TIMED step (2 events a step); the split: an untimed step with
            # every bucket's events (they stretch that step's tail by ~10 µs each)
            grad_sync["tail_ms"] = dict(tail, total_timed_step=tail_timed["total"] if tail_timed else None,
                                        split_from="untimed step at timeline level 2")
            grad_sync["bucket_timeline_ms"] = timeline
        if zero is None and args.impl == "libgsync":
            grad_sync["bucket_policy"] = log.get("bucket_policy")
            if log.get("xgmi_calibration"):
                grad_sync["xgmi_calibration"] = log["xgmi_calibration"]
        model_label = {"resnet18": "ResNet-18", "resnet50": "ResNet-50", "resnet152": "ResNet-152"}[args.model]
        line = {
            "metric": f"images/sec (node) {model_label} at 1/2/4/8 MI355X; grad-sync bus GB/s",
            "value": img_s,
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16" if args.engine == "colossal" else "bf16",
            "data": "synthetic (torch.rand 224x224 images resident in HBM, random-init weights)",
            "config": {
                "workload": (f"{args.model} synthetic 224x224 bf16 training, {args.batch} img/GPU, REFERENCE PATH for "
                             f"the ZeRO-2 config: torch FSDP(SHARD_GRAD_OP, bf16 MixedPrecision) + clip 1.0 + "
                             f"torch.optim.AdamW(fused=True) for comparison") if torch_zero else
                            (f"{args.model} synthetic 224x224 fp16-autocast training, {args.batch} img/GPU, "
                             f"REFERENCE PATH for the Colossal config: torch DDP + torch.amp.GradScaler + "
                             f"torch.optim.AdamW(fused=True) for comparison") if args.impl == "torch" and
                            args.engine == "colossal" else
                            (f"{args.model} synthetic 224x224 bf16-autocast training, {args.batch} img/GPU, "
                             f"REFERENCE PATH torch DDP + torch.optim.{'SGD' if args.optimizer == 'sgd' else 'Adam'}"
                             f"(foreach) for comparison") if args.impl == "torch" else
                            (f"{args.model} synthetic 224x224 fp16-autocast training, {args.batch} img/GPU, Colossal "
                             f"Booster(TorchDDPPlugin, mixed_precision='fp16') + HybridAdam as R:resnet/colossal/run.sh: "
                             f"libgsync DDP (fp32 buckets, GradScaler inf check fused into the unpack) + fused Adam") if
                            args.engine == "colossal" else
                            (f"{args.model} synthetic 224x224 bf16-autocast training, {args.batch} img/GPU, "
                             f"{'one hipGraph per step: ' if args.graph else ''}libgsync DDP (bucketed RCCL all-reduce overlapped with backward) + fused "
                             f"{'SGD-momentum/WD' if args.optimizer == 'sgd' else 'Adam'}") if zero is None else
                            (f"{args.model} synthetic 224x224 bf16 model training, {args.batch} img/GPU, libgsync "
                             f"{args.engine.upper()} (bf16 {'reduce-scatter' if args.engine == 'zero2' else 'all-reduce'}"
                             f" under backward, fp32 master shard, clip 1.0, fused "
                             f"{'SGD' if args.optimizer == 'sgd' else 'AdamW'}, bf16 all-gather)"),
                "engine": args.engine,
                "global_batch": args.batch * world,
                "per_gpu_batch": args.batch,
                "parallelism": f"dp{world}",
                "bucket_cap_mb": 25 if args.bucket_cap_mb is None else args.bucket_cap_mb,
                "bucket_dtype": args.bucket_dtype,
                "channels_last": not args.no_channels_last,
                "gradient_as_bucket_view": bool(args.grad_as_bucket_view),
                "impl": args.impl,
                "hipgraph": bool(args.graph),
                "optimizer_overlap": bool(args.optimizer_overlap),
                **({"rehearsal": "gloo, ranks sharing GPUs: control flow only, not a measurement"}
                   if args.pg_backend == "gloo" else {}),
                "params": n_params,
            },
            "roofline": None if args.impl == "torch" else _roofline(),
            "grad_sync": grad_sync,
            "grad_sync_kernels": kernel_rates,
            "parity": parity,
            **({"bucket_policy_ab": policy_ab} if policy_ab is not None else {}),
        **({"zero2": zero2} if zero2 is not None else {}),
        **({"colossal": colossal} if colossal is not None else {}),
            **({} if zero is None else {"zero_step_window_ms": sum(win_ms) / len(win_ms)}),
            "warmup_s": warm_s,
            "memory": {"max_allocated_GB": torch.cuda.max_memory_allocated(dev) / 2**30,
                       "reserved_GB": torch.cuda.memory_reserved(dev) / 2**30,
                       "device_total_GB": torch.cuda.get_device_properties(dev).total_memory / 2**30},
            "has_rebuilt_buckets": log.get("has_rebuilt_buckets", 0),
        }
        if leg_errors:
            line["leg_errors"] = dict(leg_errors)
        if leg_seconds:
            line["leg_seconds"] = dict(leg_seconds)
            line["leg_estimates_s"] = dict(leg_estimates, model="leg_cost(): LEG_COST_S x (ranks per GPU under gloo) "
                                                               "x batch / 256 x "
                                                               f"(1 + {LEG_GROWTH_PER_RANK} (N-1)) + per-rank "
                                                               "communicator set-up")
        if torch_ddp is not None:
            line["torch_ddp"] = torch_ddp
            if torch_ddp.get("images_per_sec"):
                line["vs_baseline"] = img_s / torch_ddp["images_per_sec"]
                line["vs_baseline_basis"] = (
                    "the reference's own GPU path timed in this run: torch DistributedDataParallel + "
                    "torch.optim.SGD(foreach) on the same model, batch, data and step "
                    "(R:resnet/pytorch_ddp/ddp_train.py:95-97); BASELINE.md publishes no number")
        return line

    # ---- after the timed region.  The headline is complete here; what follows are
    # optional legs, in order of evidence value: the tail split, the self-checked
    # parity step, the standalone collectives (bus bandwidth), the kernel rates, the
    # ZeRO-2 leg (configs[3]), the Colossal leg (configs[4]), the bucket-policy A/B.
    # --wall-budget-s (from process start) gates each: a leg whose LEG_COST_S estimate
    # does not fit what is left is skipped and named in "leg_errors" (the decision uses
    # the MAX of the ranks' clocks, so every rank skips alike); a leg that raises is
    # recorded there too instead of losing the line; a leg still running when the
    # budget ends (a hung collective) gets a watchdog that prints the line with the
    # legs completed so far and ends every rank with exit status 3.
    tail = timeline = tail_timed = None
    coll = kernel_rates = parity = policy_ab = zero2 = colossal = torch_ddp = None
    leg_errors: dict = {}
    current_leg = ["start"]

    leg_seconds: dict = {}
    budget = args.wall_budget_s

    ranks_per_gpu = -(-world // max(1, torch.cuda.device_count()))
    leg_estimates: dict = {}

    def fits(name):
        est = leg_cost(name, world, args.pg_backend, ranks_per_gpu, args.batch)
        leg_estimates[name] = round(est, 1)
        if budget <= 0:
            return True
        left = budget - coll_h.max(time.time() - T_START)
        if est <= left:
            return True
        leg_errors[name] = (f"skipped: estimated {est:.0f} s > {max(left, 0.0):.0f} s left "
                            f"of --wall-budget-s {budget:.0f}")
        if rank == 0:
            print(f"[bench] leg {name} {leg_errors[name]}", file=sys.stderr, flush=True)
        return False

    hang_leg = os.environ.get("GSYNC_BENCH_TEST_HANG_LEG")  # test hook: this leg never returns

    def leg(name, fn):
        if name != hang_leg and not fits(name):
            return None
        current_leg[0] = name
        t_leg = time.perf_counter()
        try:
            while name == hang_leg:  # tests/test_gpu_zz_bench.py: the watchdog's exit path
                time.sleep(5)
            return fn()
        except Exception as ex:  # recorded, the line still prints
            import traceback

            leg_errors[name] = repr(ex)
            print(f"[bench] leg {name} failed: {ex!r}\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            return None
        finally:
            leg_seconds[name] = round(time.perf_counter() - t_leg, 2)

    watchdog = None
    if budget > 0:
        import threading

        def expire():
            if rank == 0:
                try:
                    ln = make_line()
                except Exception as ex:  # the headline alone, whatever else failed
                    ln = {"metric": "images/sec (node) ResNet-50 at 1/2/4/8 MI355X; grad-sync bus GB/s",
                          "value": img_s, "unit": "images/sec", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
                          "config": {"workload": f"{args.model} synthetic 224x224 training, {args.batch} img/GPU",
                                     "parallelism": f"dp{world}", "global_batch": args.batch * world},
                          "line_error": repr(ex)}
                ln["legs_incomplete"] = {"leg": current_leg[0], "wall_budget_s": budget}
                print(json.dumps(ln), flush=True)
            print(f"[bench] rank {rank}: leg {current_leg[0]} still running at the {budget:.0f} s wall budget: "
                  "exiting with status 3", file=sys.stderr, flush=True)
            os._exit(3)

        # a leg only starts when its estimate fits the budget: one that is still running
        # 30 s past it overran its estimate several times over (a hang), not a slow box
        watchdog = threading.Timer(max(1.0, T_START + budget + 30.0 - time.time()), expire)
        watchdog.daemon = True
        watchdog.start()

    def tail_leg():
        nonlocal tail, timeline, tail_timed, comm_ms
        if zero is None and args.impl == "libgsync" and not args.graph:
            # timed steps ran at timeline level 1: two events per step, the tail total
            # (last bucket ready -> every bucket chain done) of the last timed step
            tail_timed = ddp.tail_ms()
            # the split (queue / pack / collective / unpack per bucket) needs ~4 events a
            # bucket, ~10 µs each on the exposed tail: read it from untimed steps at level 2
            ddp.set_timeline(2)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            comm_ms = [m for m in ddp.bucket_comm_ms() if m >= 0]  # per bucket, HIP events on the comm stream
            tail = ddp.tail_ms()
            timeline = ddp.bucket_timeline_ms()
            ddp.set_timeline(1)
            opt.kernel_ms()  # drop the untimed steps' launches

    leg("tail_split", tail_leg)

    if args.parity and args.impl == "libgsync" and not args.graph:
        from distributed_training_amd import parity as PC

        if zero is None and args.engine == "colossal":
            def fwd_bwd():
                booster.backward(ccrit(cmodel(x), y), opt_w)

            parity = leg("parity", lambda: PC.ddp_parity_step(ddp, opt_w, fwd_bwd))
        elif zero is None:
            def fwd_bwd():
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = crit(ddp(x), y)
                loss.backward()

            parity = leg("parity", lambda: PC.ddp_parity_step(ddp, opt, fwd_bwd))
        else:
            def fwd_bwd():
                crit(ddp(x).float(), y).backward()

            parity = leg("parity", lambda: PC.zero_parity_step(zero, fwd_bwd))
        if rank == 0:
            print(f"[bench] parity: {json.dumps(parity)}", file=sys.stderr, flush=True)

    if args.impl == "libgsync" and (args.collective_bench == 1 or (args.collective_bench == -1 and world > 1)):
        coll = leg("collective_bench", lambda: collective_bench(ddp, zero, world))
    if args.impl == "libgsync" and args.kernel_rates:
        # rank 0 measures; the others wait in the next leg's (or the end's) collective
        kernel_rates = leg("kernel_rates", lambda: grad_sync_kernel_rates(
            [p for p in model.parameters() if p.requires_grad] if zero is None else zero.params, dev,
            comm=_engine_comm(ddp, zero), world=world) if rank == 0 else None)

    want_zero = args.zero_leg != 0
    if want_zero and args.impl == "libgsync" and args.engine == "ddp" and not args.graph:
        zero2 = leg("zero2", lambda: zero2_leg(args, world, rank, dev, coll_h))
        if rank == 0 and zero2 is not None:
            print(f"[bench] zero2 leg: {zero2['images_per_sec']:.1f} images/s, parity {zero2['parity'].get('ok')}",
                  file=sys.stderr, flush=True)
    want_col = args.colossal_leg != 0
    if want_col and args.impl == "libgsync" and args.engine == "ddp" and not args.graph:
        colossal = leg("colossal", lambda: colossal_leg(args, world, rank, dev, coll_h,
                                                        batch=min(128, args.batch)))
        if rank == 0 and colossal is not None:
            print(f"[bench] colossal leg: {colossal['images_per_sec']:.1f} images/s, "
                  f"parity {colossal['parity'].get('ok')}", file=sys.stderr, flush=True)
    want_ab = args.policy_ab == 1 or (args.policy_ab == -1 and world > 1)
    if (want_ab and args.impl == "libgsync" and args.engine == "ddp" and not args.graph
            and not args.optimizer_overlap):
        # after every reading of the headline DDP above: it is closed here
        policy_ab = leg("bucket_policy_ab", lambda: bucket_policy_ab(model, opt, ddp, x, y, crit, world, dev, args))
        if rank == 0 and policy_ab is not None:
            print(f"[bench] bucket policy A/B: decision {policy_ab['decision']}", file=sys.stderr, flush=True)
    # the torch legs come after the policy A/B: at N > 1 the A/B decides row N1, the
    # torch legs only set vs_baseline, so a tight budget skips them first
    if args.torch_leg != 0 and args.impl == "libgsync" and args.engine == "ddp" and not args.graph:
        torch_ddp = leg("torch_ddp", lambda: torch_ddp_leg(args, world, rank, dev, mf))
        if rank == 0 and torch_ddp is not None:
            print(f"[bench] torch DDP leg: {torch_ddp['images_per_sec']:.1f} images/s "
                  f"(libgsync {img_s:.1f})", file=sys.stderr, flush=True)
        # configs[4] on torch alone, beside its libgsync leg.  (configs[3]'s torch FSDP
        # SHARD_GRAD_OP step read 108-110 ms a step inside this process against 81.5 ms
        # standalone — r6d, r6f against r6e, cause not found — so it is timed standalone:
        # scripts/r6e_zero2_vs_fsdp.sh)
        if colossal is not None and colossal.get("images_per_sec"):
            tc = leg("torch_colossal", lambda: torch_colossal_leg(args, world, rank, dev, batch=min(128, args.batch)))
            if tc is not None:
                colossal["torch"] = tc
                colossal["vs_torch"] = colossal["images_per_sec"] / tc["images_per_sec"]
    current_leg[0] = "done"
    if watchdog is not None:
        watchdog.cancel()
    # tear down what the run created before the process group goes, as the reference
    # does (R:resnet/pytorch_ddp/ddp_train.py:87-88,105): the engines, then libgsync's
    # communicators
    if args.impl == "libgsync":
        for eng in (zero, ddp, getattr(ddp, "module", None)):
            if isinstance(eng, (D.DistributedDataParallel,)) or type(eng).__name__ == "ZeroDataParallel":
                try:
                    eng.close()
                except Exception as ex:  # the line still prints
                    print(f"[bench] close: {ex!r}", file=sys.stderr, flush=True)
        D.destroy_communicators()

    # free the engines (reference cycles hold the process group) before the teardown:
    # a gloo worker thread dropping a Python tensor during interpreter finalization
    # ends in std::terminate
    import gc

    gc.collect()
    if rank != 0:
        dist.destroy_process_group()
        return

    line = make_line()
    if args.cpu_baseline and world == 1:
        from oracle.cpu_ddp_baseline import cpu_model_name, run as cpu_run

        hc = _host_cores()
        cores = hc["cores_used"]
        # leg 1 (the headline unit): the reference's torch-DDP/gloo path on this workload's model at 224x224;
        # leg 2: BASELINE configs[0], the reference's own workload (ResNet-18 CIFAR, 100 img/rank, ws=2)
        cb = cpu_run(model=args.model, batch=16, ws=2, cores=cores, steps=5, warmup=1, port=_free_port())
        c1 = cpu_run(model="resnet18", batch=100, ws=2, cores=cores, steps=10, warmup=2, port=_free_port())
        line["cpu_baseline"] = {
            "value": cb["images_per_sec"],
            "unit": "images/sec",
            "cores": cb["cores"],
            "cores_available": hc,
            "cpu_model": cpu_model_name(),
            "kind": "port",
            "gloo_allreduce_busbw_GBps": cb["gloo_allreduce_busbw_GBps"],
            "gloo_allreduce_bytes": cb["gloo_allreduce_bytes"],
            "sample": f"torch DDP+gloo {args.model} 224x224, Adam(lr=1e-3*ws), ws=2 x 16 img/rank, "
                      f"1 warmup + 5 timed steps (restates R:resnet/pytorch_ddp/ddp_train.py:79-114 on CPU)",
            "config0_resnet18_cifar": {
                "value": c1["images_per_sec"], "unit": "images/sec", "cores": c1["cores"],
                "gloo_allreduce_busbw_GBps": c1["gloo_allreduce_busbw_GBps"],
                "sample": "torch DDP+gloo resnet18 32x32 10 classes, Adam(lr=1e-3*ws), ws=2 x 100 img/rank "
                          "(R:resnet/pytorch_ddp/ddp_train.py:95,97,110-111), 2 warmup + 10 timed steps"},
        }
    print(json.dumps(line), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
    import gc

    gc.collect()  # main()'s engines are unreachable now: their process group goes before finalization
