"""Roofline microbenchmark of the grad-sync kernels at BASELINE sizes, beside
the reference's GPU path for the same work (torch ops on the same device).

For ResNet-50 / ResNet-152 parameter sets (real per-tensor shapes) it times,
with HIP events on the stream each kernel is launched on (libgsync rows: the
plan launch timer, events recorded by the library around each kernel; every
row also `batched_*`: the same launches back to back between one event pair):

  libgsync                         reference GPU path (torch 2.10 on ROCm)
  pack fp32 (x 1/ws)   8 B/param    per-param  torch.mul(grad, 1/ws, out=bucket_view)  (Reducer mark_variable_ready_dense)
  pack fp32->bf16      6 B/param    per-param  bucket_view.copy_(grad.mul(1/ws))
  unpack fp32          8 B/param    per-param  grad.copy_(bucket_view)                 (copy_bucket_to_grad)
  SGD momentum+wd     20 B/param    torch.optim.SGD foreach=True  step
  Adam                28 B/param    torch.optim.Adam foreach=True step
  sq-norm              4 B/param    torch._foreach_norm + stack/norm (clip_grad_norm_)

Working sets are replicated `--replicas` times so the timed data exceeds the
256 MiB Infinity Cache (true HBM rates).  Prints one JSON object per kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

HBM_PEAK = 8000.0


_LAST = {}


def timeit_plan(plan, fn, iters=20, warmup=3):
    """libgsync launches: the plan launch timer (HIP events recorded by the
    library right around each kernel on its stream)."""
    _LAST["fn"] = fn
    for _ in range(warmup):
        fn()
    plan.timer_enable(iters)
    for _ in range(iters):
        fn()
    ts = sorted(plan.timer_read())
    plan.timer_enable(0)
    return ts[len(ts) // 2], sum(ts) / len(ts)


def timeit_batched(fn, iters=20):
    """`iters` back-to-back launches between ONE pair of HIP events on the
    current stream (launch gaps included, no per-launch event cost)."""
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    _LAST["fn"] = fn
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2], sum(ts) / len(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--skip-torch", action="store_true")
    ap.add_argument("--tag", default=os.environ.get("GSYNC_LIB", "libgsync").split("/")[-1])
    args = ap.parse_args()
    from distributed_training_amd.multi_tensor import TensorListPlan
    from distributed_training_amd.resnet import MODELS

    dev = torch.device("cuda", 0)
    shapes = [p.shape for p in MODELS[args.model]().parameters()] * args.replicas
    n = sum(torch.Size(s).numel() for s in shapes)
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda scale=1.0: [torch.randn(s, device=dev, generator=g) * scale for s in shapes]  # noqa: E731
    params, grads, bufs = mk(), mk(0.01), mk(0.01)
    ms, vs = mk(0.01), [x.abs() for x in mk(1e-4)]
    plan = TensorListPlan([torch.Size(s).numel() for s in shapes], dev, align=64)
    flat = torch.zeros(plan.flat_numel, device=dev)
    flat16 = torch.zeros(plan.flat_numel, device=dev, dtype=torch.bfloat16)
    offs = plan.offsets
    views = [flat[o:o + torch.Size(s).numel()].view(s) for o, s in zip(offs, shapes)]
    views16 = [flat16[o:o + torch.Size(s).numel()].view(s) for o, s in zip(offs, shapes)]
    out = []

    last_fn = _LAST

    def rec(name, nbytes, ms_med, ms_avg, impl):
        gbs = nbytes / (ms_avg * 1e-3) / 1e9
        row = {"kernel": name, "impl": impl, "model": args.model, "replicas": args.replicas, "params": n,
               "tag": args.tag, "task_units": plan.task_units, "n_tasks": plan.n_tasks,
               "alg_bytes": nbytes, "median_ms": ms_med, "avg_ms": ms_avg, "GBps": gbs, "frac_of_8TBps": gbs / HBM_PEAK}
        if "fn" in last_fn:  # the same launches, batched between one event pair
            bms = timeit_batched(last_fn.pop("fn"), args.iters)
            bgbs = nbytes / (bms * 1e-3) / 1e9
            row.update({"batched_avg_ms": bms, "batched_GBps": bgbs, "batched_frac_of_8TBps": bgbs / HBM_PEAK})
        out.append(row)
        print(json.dumps(row), flush=True)

    plan.set_ptrs(1, grads)
    plan.set_ptrs(2, grads)
    rec("pack_f32", 8 * n, *timeit_plan(plan, lambda: plan.pack(1, torch.float32, flat, 0.125, 1), args.iters), "libgsync")
    rec("pack_f32_to_bf16", 6 * n, *timeit_plan(plan, lambda: plan.pack(1, torch.float32, flat16, 0.125, 1), args.iters), "libgsync")
    rec("unpack_f32", 8 * n, *timeit_plan(plan, lambda: plan.unpack(flat, 2, torch.float32), args.iters), "libgsync")
    sq = torch.zeros(1, device=dev)
    rec("unpack_f32+sqnorm", 8 * n, *timeit_plan(plan, lambda: plan.unpack(flat, 2, torch.float32, sqnorm=sq), args.iters), "libgsync")
    rec("sqnorm_f32", 4 * n, *timeit_plan(plan, lambda: plan.sqnorm(1, torch.float32, sq), args.iters), "libgsync")
    # the update kernels run on an update plan, as FusedSGD / FusedAdam build it
    from distributed_training_amd.multi_tensor import update_task_units

    plan = TensorListPlan([torch.Size(s).numel() for s in shapes], dev, task_units=update_task_units(dev))
    plan.set_ptrs(0, params)
    plan.set_ptrs(1, grads)
    plan.set_ptrs(2, bufs)
    rec("sgd_momentum_wd", 20 * n, *timeit_plan(plan, lambda: plan.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False),
                                                args.iters), "libgsync")
    plan.set_ptrs(2, ms)
    plan.set_ptrs(3, vs)
    rec("adam", 28 * n, *timeit_plan(plan, lambda: plan.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5),
                                     args.iters), "libgsync")
    if not args.skip_torch:
        inv = 1.0 / 8

        def t_pack():
            for gr, v in zip(grads, views):
                torch.mul(gr, inv, out=v)

        def t_pack16():
            for gr, v in zip(grads, views16):
                v.copy_(gr.mul(inv))

        def t_unpack():
            for gr, v in zip(grads, views):
                gr.copy_(v)

        rec("pack_f32", 8 * n, *timeit(t_pack, args.iters), "torch per-param (Reducer)")
        rec("pack_f32_to_bf16", 6 * n, *timeit(t_pack16, args.iters), "torch per-param (Reducer)")
        rec("unpack_f32", 8 * n, *timeit(t_unpack, args.iters), "torch per-param (Reducer)")
        rec("sqnorm_f32", 4 * n, *timeit(lambda: torch.linalg.vector_norm(torch.stack(torch._foreach_norm(grads))),
                                         args.iters), "torch _foreach_norm")
        ps = [torch.nn.Parameter(p.clone()) for p in params]
        for p, gr in zip(ps, grads):
            p.grad = gr
        sgd = torch.optim.SGD(ps, lr=1e-6, momentum=0.9, weight_decay=1e-4, foreach=True)
        rec("sgd_momentum_wd", 20 * n, *timeit(sgd.step, args.iters), "torch.optim.SGD foreach")
        adam = torch.optim.Adam(ps, lr=1e-6, foreach=True)
        rec("adam", 28 * n, *timeit(adam.step, args.iters), "torch.optim.Adam foreach")
        fadam = torch.optim.Adam(ps, lr=1e-6, fused=True)
        rec("adam", 28 * n, *timeit(fadam.step, args.iters), "torch.optim.Adam fused")


if __name__ == "__main__":
    main()
