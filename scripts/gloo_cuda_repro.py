"""Minimal reproduction of the 4-rank gloo rehearsal stall:
ranks sharing one GPU issue several async gloo all-reduces of CUDA buffers
(the sizes of ResNet-50's rebuilt buckets) while their default stream is
still busy, then wait on them in order — what the bench's external-collective
path does in warm-up step 1.  No libgsync involved.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29611 scripts/gloo_cuda_repro.py

MODE=main: issue from the main thread; MODE=hook: from post-accumulate-grad
hooks on the autograd thread (as ddp.py); MODE=cpu: stage each bucket through
an explicit D2H copy and all-reduce the host copy (gloo's CPU path).
"""
import faulthandler
import os
import sys
import time

import torch
import torch.distributed as dist

faulthandler.dump_traceback_later(float(os.environ.get("TB_S", "45")), repeat=True)
rank = int(os.environ["RANK"])
ws = int(os.environ["WORLD_SIZE"])
mode = os.environ.get("MODE", "main")
iters = int(os.environ.get("ITERS", "4"))
busy = int(os.environ.get("BUSY", "12"))
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("gloo")
sizes = [2049000, 7875584, 6563840, 6637568, 2431040]  # ResNet-50's rebuilt fp32 buckets (elements)
bufs = [torch.zeros(n, device=dev) for n in sizes]
a = torch.randn(4096, 4096, device=dev)
log = open(os.path.join(os.environ.get("OUT", "gpurun_out"), f"repro_{mode}_ws{ws}_r{rank}.log"), "w")


def say(*x):
    print(f"[r{rank}]", *x, file=log, flush=True)
    if rank == 0:
        print(f"[r{rank}]", *x, file=sys.stderr, flush=True)


def spin():
    global a
    for _ in range(busy):
        a = torch.tanh(a @ a * 1e-3)


if mode == "hook":
    params = [torch.nn.Parameter(torch.zeros(n, device=dev)) for n in sizes]
    works = []

    def make_hook(i):
        def hook(p):
            bufs[i].copy_(p.grad)
            say(f"enqueue {i}")
            works.append(dist.all_reduce(bufs[i], async_op=True))
        return hook

    for i, p in enumerate(params):
        p.register_post_accumulate_grad_hook(make_hook(i))

for it in range(iters):
    t0 = time.time()
    for b in bufs:
        b.fill_(float(rank + 1))
    if mode == "hook":
        works.clear()
        w = torch.randn(4096, 4096, device=dev, requires_grad=True)
        loss = 0.0
        for i, p in enumerate(params):  # each param's grad is ready after a chunk of backward compute
            h = torch.tanh(w @ w * 1e-3)
            for _ in range(busy // 4):
                h = torch.tanh(h @ h * 1e-3)
            loss = loss + (p * h.mean()).sum()
        loss.backward()
        for i, wk in enumerate(works):
            say(f"wait {i}")
            wk.wait()
    elif mode == "cpu":
        hosts = []
        for i, b in enumerate(bufs):
            spin()
            h = b.to("cpu", non_blocking=False)
            hosts.append((h, dist.all_reduce(h, async_op=True)))
        for i, ((h, wk), b) in enumerate(zip(hosts, bufs)):
            say(f"wait {i}")
            wk.wait()
            b.copy_(h)
    else:
        works = []
        for i, b in enumerate(bufs):
            spin()
            say(f"enqueue {i}")
            works.append(dist.all_reduce(b, async_op=True))
        for i, wk in enumerate(works):
            say(f"wait {i}")
            wk.wait()
    torch.cuda.synchronize()
    want = float(sum(range(1, ws + 1)))
    ok = all(bool((b == want).all()) for b in bufs) if mode != "hook" else True
    say(f"iter {it}: {time.time() - t0:.2f}s ok={ok}")
faulthandler.cancel_dump_traceback_later()
dist.destroy_process_group()
say("done")
