"""Diagnostic: libgsync's communicator collectives vs stream order — is the
work queued before a collective on the caller's stream (the output's fill)
ordered before it?  `side` runs on a created stream instead of the default
one (handle 0, which the ABI once mistook for "the comm stream").  Prints
per case whether the output is exact."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from distributed_training_amd.comm import get_communicator  # noqa: E402

c = get_communicator(None, torch.device("cuda", 0))
side = torch.cuda.Stream()
if len(sys.argv) > 1 and sys.argv[1] == "side":  # a created (non-null) stream instead of the default one
    torch.cuda.set_stream(side)
cur = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
print("stream handle", cur(), flush=True)
for n in (1 << 20, 1 << 22, 1 << 24):
    for dt in (torch.float32, torch.int32, torch.bfloat16):
        x = (torch.arange(n, device="cuda") % 1000 + 1).to(dt)
        res = {}
        for op in ("ag", "ar", "rs", "bc"):
            for mode in ("nosync", "sync_before"):
                out = torch.zeros_like(x)
                if mode == "sync_before":
                    torch.cuda.synchronize()
                if op == "ag":
                    c.all_gather(x, out, stream=cur())
                elif op == "ar":
                    c.all_reduce(x, out=out, stream=cur())
                elif op == "rs":
                    c.reduce_scatter(x, out, stream=cur())
                else:
                    out.copy_(x)
                    out2 = out
                    c.broadcast(out2, root=0, stream=cur())
                torch.cuda.synchronize()
                res[f"{op}/{mode}"] = int((out == x).sum()) == n
        print(n, dt, res, flush=True)
dist.destroy_process_group()
