"""The end of backward in a DDP step, kernel by kernel: what every queue runs
from 150 µs before backward's last kernel to the end of the step's update.

    rocprofv3 --kernel-trace -f csv -d <dir> -o tail -- python3 scripts/tail_trace.py run
    python3 scripts/tail_trace.py analyze <kernel_trace.csv> > tail.jsonl

`run`: ResNet-50, batch 256, bf16 autocast + channels_last, libgsync DDP +
FusedSGD, as bench.py's headline step, 8 steps.  `analyze`: for each of the
last three steps, backward's last kernel (the last kernel that is neither
libgsync's nor RCCL's before the step's SGD) is t = 0; every kernel overlapping
[-150 µs, SGD end] with its queue, start / end (µs) and a short name.
"""
import csv
import json
import os
import re
import sys


def run():
    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # as bench.py: an nccl process group; libgsync brings up its own RCCL communicator
    torch.distributed.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1)
    model = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (256,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()
    for _ in range(8):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    torch.cuda.synchronize()
    torch.distributed.destroy_process_group()


def short(name):
    m = re.search(r"chunk_kernel<gs::\(anonymous namespace\)::(\w+)<", name)
    if m:
        return "gs:" + m.group(1)
    if "nccl" in name.lower():
        return "rccl:" + name.split("(")[0][-40:]
    return name.split("(")[0][:60]


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
    sgd = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "gs:SgdOp"]
    for si in sgd[-3:]:
        s_end = int(rows[si]["End_Timestamp"])
        bwd = None
        for j in range(si - 1, -1, -1):
            n = short(rows[j]["Kernel_Name"])
            if not (n.startswith("gs:") or n.startswith("rccl:")):
                bwd = j
                break
        t0 = int(rows[bwd]["End_Timestamp"])
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e >= t0 - 150_000 and s <= s_end:
                print(json.dumps({"step_sgd_index": si, "queue": r.get(qkey) if qkey else None,
                                  "kernel": short(r["Kernel_Name"]), "start_us": (s - t0) / 1e3,
                                  "end_us": (e - t0) / 1e3, "dur_us": (e - s) / 1e3}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyze(sys.argv[2])
