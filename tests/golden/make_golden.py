"""Generate the golden fixtures under tests/golden/ (run in the build
container, which has /root/reference; the outputs are plain data files).

What runs is the REFERENCE's own training step: ``train_epoch`` imported from
R:resnet/pytorch_ddp/ddp_train.py:52-75 (with a local torchvision stand-in on
sys.path, tests/golden/_shim), driving torch's DistributedDataParallel exactly
as R:resnet/pytorch_ddp/ddp_train.py:95-98 builds it, except: backend gloo on
CPU (ddp_setup :79-85 hard-codes nccl + cuda), synthetic batches (CIFAR10
needs the network), and a small BasicBlock[1,1,1,1] width-4 ResNet so full
tensors fit in a fixture.  Optimizers: the reference's Adam(lr=1e-3*ws)
(:97,:110) and the north-star SGD(lr=0.1, momentum=0.9, wd=1e-4).

Outputs
  ddp_<opt>_ws<N>.npz   init params, per-rank batches, per-rank local grads of
                        step 1, averaged grads and params after each step,
                        per-rank BN buffers after the last step
  ddp_bf16hook_ws2.npz  averaged grads with torch's bf16_compress_hook
  r18_digest_ws2.json   full ResNet-18/CIFAR: per-tensor digests of the
                        averaged grads and post-step weights (Adam, 2 steps)
  buckets.json          torch's bucket assignment (init + rebuilt, fp32/bf16)
                        and rebuilt_bucket_sizes for ResNet-18/50/152
  optim.npz             single-step torch SGD / Adam / AdamW / clip_grad_norm_
  state_dict_keys.json  DDP state_dict keys of the ResNets (module. prefix)

Usage: python tests/golden/make_golden.py   (about a minute on 8 cores)
"""
from __future__ import annotations

import copy
import importlib.util
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DDP = "/root/reference/resnet/pytorch_ddp/ddp_train.py"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(HERE, "_shim"))

from distributed_training_amd.resnet import ResNet, BasicBlock, resnet18, resnet50, resnet152  # noqa: E402

BATCH = 4
STEPS = 3
MICRO_WIDTH = 4


def micro():
    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=MICRO_WIDTH)


def load_reference_trainer():
    spec = importlib.util.spec_from_file_location("ref_ddp_train", REF_DDP)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_batches(rank, steps, batch, hw=32, classes=10):
    g = torch.Generator().manual_seed(1234 + rank)
    return [(torch.rand(batch, 3, hw, hw, generator=g), torch.randint(0, classes, (batch,), generator=g))
            for _ in range(steps)]


def make_opt(kind, params, ws):
    base = torch.optim.Adam if kind == "adam" else torch.optim.SGD
    kw = dict(lr=1e-3 * ws) if kind == "adam" else dict(lr=0.1, momentum=0.9, weight_decay=1e-4)

    class Recording(base):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.grads, self.params = [], []

        def step(self, closure=None):
            self.grads.append([p.grad.detach().clone() for p in self.param_groups[0]["params"]])
            out = super().step(closure)
            self.params.append([p.detach().clone() for p in self.param_groups[0]["params"]])
            return out

    return Recording(params, foreach=False, **kw)


def _init(rank, ws, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    torch.set_num_threads(max(1, 8 // ws))


def ddp_worker(rank, ws, kind, port, out_path, hook):
    _init(rank, ws, port)
    ref = load_reference_trainer()
    from torch.nn.parallel import DistributedDataParallel as DDP

    torch.manual_seed(100 + rank)  # different per rank: DDP's init broadcast must fix it
    model = micro()
    ddp = DDP(model)
    if hook:
        from torch.distributed.algorithms.ddp_comm_hooks.default_hooks import bf16_compress_hook
        ddp.register_comm_hook(None, bf16_compress_hook)
    init = [p.detach().clone() for p in model.parameters()]
    batches = make_batches(rank, STEPS, BATCH)
    # local (un-synchronised) grads of step 1 from an identical replica
    rep = micro()
    rep.load_state_dict(model.state_dict())
    rep.train()
    nn.CrossEntropyLoss()(rep(batches[0][0]), batches[0][1]).backward()
    local = [p.grad.detach().clone() for p in rep.parameters()]
    opt = make_opt(kind, ddp.parameters(), ws)
    ref.train_epoch(0, 1, ddp, opt, nn.CrossEntropyLoss(), batches, "cpu")
    bufs = [b.detach().clone() for b in model.buffers()]
    payload = dict(local=local, batches=batches, bufs=bufs, grads=opt.grads, params=opt.params, init=init,
                   rebuilt=ddp._get_ddp_logging_data().get("rebuilt_bucket_sizes", []))
    gathered = [None] * ws
    dist.all_gather_object(gathered, payload)
    if rank == 0:
        names = [n for n, _ in model.named_parameters()]
        bnames = [n for n, _ in model.named_buffers()]
        arrs = {"param_names": np.array(names), "buffer_names": np.array(bnames),
                "ws": np.array(ws), "steps": np.array(STEPS)}
        for i, t in enumerate(init):
            arrs[f"init/{i}"] = t.numpy()
        for r in range(ws):
            pr = gathered[r]
            for s, (x, y) in enumerate(pr["batches"]):
                arrs[f"x/{r}/{s}"] = x.numpy()
                arrs[f"y/{r}/{s}"] = y.numpy()
            for i, t in enumerate(pr["local"]):
                arrs[f"local/{r}/{i}"] = t.numpy()
            for i, t in enumerate(pr["bufs"]):
                arrs[f"buf/{r}/{i}"] = t.numpy()
        for s in range(len(opt.grads)):
            for i, t in enumerate(opt.grads[s]):
                arrs[f"grad/{s}/{i}"] = t.numpy()
            for i, t in enumerate(opt.params[s]):
                arrs[f"param/{s}/{i}"] = t.numpy()
        # every rank must hold the same averaged grads
        for r in range(1, ws):
            for a, b in zip(gathered[r]["grads"][0], opt.grads[0]):
                assert torch.equal(a, b), "ranks disagree on averaged grads"
        np.savez_compressed(out_path, **arrs)
    dist.destroy_process_group()


def digest(t: torch.Tensor):
    x = t.detach().double().reshape(-1)
    idx = torch.linspace(0, x.numel() - 1, steps=min(64, x.numel())).long()
    return {"sum": x.sum().item(), "sumsq": (x * x).sum().item(), "maxabs": x.abs().max().item(),
            "samples": x[idx].tolist(), "idx": idx.tolist()}


def r18_worker(rank, ws, port, out_path):
    _init(rank, ws, port)
    ref = load_reference_trainer()
    from torch.nn.parallel import DistributedDataParallel as DDP

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    ddp = DDP(model)
    init_digest = [digest(p) for p in model.parameters()]
    batches = make_batches(rank, 2, 100)  # batch_size 100 per rank (R:ddp_train.py:111)
    opt = make_opt("adam", ddp.parameters(), ws)
    ref.train_epoch(0, 1, ddp, opt, nn.CrossEntropyLoss(), batches, "cpu")
    if rank == 0:
        out = {"ws": ws, "batch": 100, "seed_model": 0, "seed_data": "1234+rank", "optimizer": "Adam(lr=1e-3*ws)",
               "param_names": [n for n, _ in model.named_parameters()],
               "init": init_digest,
               "grads": [[digest(g) for g in step] for step in opt.grads],
               "params": [[digest(p) for p in step] for step in opt.params]}
        with open(out_path, "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


def bucket_worker(rank, ws, port, out_path):
    _init(rank, ws, port)
    from torch.nn.parallel import DistributedDataParallel as DDP

    out = {}
    for name, fn, classes, hw in (("resnet18", resnet18, 10, 32), ("resnet50", resnet50, 1000, 64),
                                  ("resnet152", resnet152, 1000, 64)):
        for dtype in (torch.float32, torch.bfloat16):
            torch.manual_seed(0)
            model = fn(num_classes=classes).to(dtype)
            params = [p for p in model.parameters()]
            order = []
            for i, p in enumerate(params):
                p.register_post_accumulate_grad_hook(lambda _p, i=i: order.append(i))
            ddp = DDP(model)
            for it in range(2):
                x = torch.rand(2, 3, hw, hw).to(dtype)
                ddp(x).float().sum().backward()
                if it == 0:
                    first_order = list(order)
                ddp.zero_grad()
            log = ddp._get_ddp_logging_data()
            init_assign, init_limits = dist._compute_bucket_assignment_by_size(params, [2**62], [False] * len(params))
            rebuilt, _ = dist._compute_bucket_assignment_by_size(
                # Reducer::rebuild_buckets passes rebuilt_params_ (tensors in ready order)
                # together with rebuilt_param_indices_
                [params[i] for i in first_order], [dist._DEFAULT_FIRST_BUCKET_BYTES, 25 * 1024 * 1024],
                [False] * len(params), first_order)
            out[f"{name}/{str(dtype).split('.')[-1]}"] = {
                "numels": [p.numel() for p in params],
                "element_size": params[0].element_size(),
                "ready_order": first_order,
                "init_assignment": [list(map(int, b)) for b in init_assign],
                "rebuilt_assignment": [list(map(int, b)) for b in rebuilt],
                "rebuilt_bucket_sizes": list(map(int, log.get("rebuilt_bucket_sizes", []))),
                "bucket_sizes": list(map(int, log.get("bucket_sizes", []))),
            }
            del ddp
    with open(out_path, "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


def optim_fixture(path):
    g = torch.Generator().manual_seed(7)
    sizes = [1, 3, 5, 64, 127, 1000, 4099]
    arrs = {"sizes": np.array(sizes)}
    cases = {
        "sgd_plain": (torch.optim.SGD, dict(lr=0.1)),
        "sgd_mom_wd": (torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
        "sgd_nesterov": (torch.optim.SGD, dict(lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-4)),
        "sgd_damp": (torch.optim.SGD, dict(lr=0.05, momentum=0.8, dampening=0.3)),
        "adam_ref": (torch.optim.Adam, dict(lr=2e-3)),  # R:ddp_train.py:97,110 at ws=2
        "adam_wd": (torch.optim.Adam, dict(lr=1e-3, betas=(0.8, 0.999), eps=1e-8, weight_decay=3e-7)),
        "adamw_ds": (torch.optim.AdamW, dict(lr=1e-3, betas=(0.8, 0.999), eps=1e-8, weight_decay=3e-7)),
    }
    for name, (cls, kw) in cases.items():
        ps = [torch.randn(n, generator=g) for n in sizes]
        gs_steps = [[torch.randn(n, generator=g) * 0.1 for n in sizes] for _ in range(3)]
        for i, p in enumerate(ps):
            arrs[f"{name}/p0/{i}"] = p.numpy().copy()
        params = [nn.Parameter(p.clone()) for p in ps]
        opt = cls(params, foreach=False, **kw)
        for s in range(3):
            for i, (p, gg) in enumerate(zip(params, gs_steps[s])):
                p.grad = gg.clone()
                arrs[f"{name}/g/{s}/{i}"] = gg.numpy().copy()
            opt.step()
            for i, p in enumerate(params):
                arrs[f"{name}/p/{s}/{i}"] = p.detach().numpy().copy()
        arrs[f"{name}/kw"] = np.array(json.dumps(kw))
    # clip_grad_norm_
    for name, scale in (("clip_big", 10.0), ("clip_small", 1e-3)):
        gs_ = [torch.randn(n, generator=g) * scale for n in sizes]
        params = [nn.Parameter(torch.zeros(n)) for n in sizes]
        for i, (p, gg) in enumerate(zip(params, gs_)):
            p.grad = gg.clone()
            arrs[f"{name}/g/{i}"] = gg.numpy().copy()
        norm = torch.nn.utils.clip_grad_norm_(params, max_norm=1.0, foreach=False)
        arrs[f"{name}/norm"] = norm.numpy()
        for i, p in enumerate(params):
            arrs[f"{name}/out/{i}"] = p.grad.numpy().copy()
    np.savez_compressed(path, **arrs)


def keys_fixture(path):
    out = {}
    for name, fn, classes in (("resnet18", resnet18, 10), ("resnet50", resnet50, 1000), ("resnet152", resnet152, 1000)):
        out[name] = ["module." + k for k in fn(num_classes=classes).state_dict().keys()]
    with open(path, "w") as f:
        json.dump(out, f)


def spawn(fn, ws, *args):
    mp.spawn(fn, args=(ws,) + args, nprocs=ws, join=True)


def main():
    port = 29600
    for kind, ws in (("sgd", 2), ("adam", 2), ("sgd", 4)):
        port += 1
        spawn(ddp_worker, ws, kind, port, os.path.join(HERE, f"ddp_{kind}_ws{ws}.npz"), False)
        print("wrote", kind, ws, flush=True)
    port += 1
    spawn(ddp_worker, 2, "sgd", port, os.path.join(HERE, "ddp_bf16hook_ws2.npz"), True)
    port += 1
    spawn(r18_worker, 2, port, os.path.join(HERE, "r18_digest_ws2.json"))
    port += 1
    spawn(bucket_worker, 1, port, os.path.join(HERE, "buckets.json"))
    optim_fixture(os.path.join(HERE, "optim.npz"))
    keys_fixture(os.path.join(HERE, "state_dict_keys.json"))
    print("done")


if __name__ == "__main__":
    main()
