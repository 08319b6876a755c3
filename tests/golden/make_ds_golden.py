"""Generate tests/golden/ds_harness_ws2.npz by driving the DeepSpeed shim with
the REFERENCE's own DeepSpeed harness (run in the build container, which has
/root/reference; the output is plain data).

What runs unchanged from R:resnet/deepspeed/deepspeed_train.py:
  * add_argument() (:27-129) — its argparse surface plus
    deepspeed.add_config_arguments (:125), parsing
    `--deepspeed --stage {0,2} --dtype {bf16,fp32}`;
  * train_epoch() (:133-158) — model.train(), the tqdm loop over the engine's
    loader, `model(images)` on the raw module, engine.backward / engine.step.
What is restated: the __main__ block (:161-258, it hard-codes torchvision's
CIFAR10 download and `.cuda()`): the same ds_config values (:172-220), a
synthetic CIFAR-shaped dataset, the width-4 BasicBlock[1,1,1,1] ResNet of the
other fixtures, CPU/gloo world size 2, `deepspeed.init_distributed()` first as
:168 does.  `deepspeed` / `torchvision` resolve to libgsync's shims
(distributed_training_amd/compat/shims, tests/golden/_shim): DeepSpeed itself
is not installed, so this pins the reference harness's CALL SURFACE and the
shim's numerics as driven by it (DeepSpeed's own numerics stay unpinned).

Recorded per (stage, dtype): every step's loss on each rank (the criterion
the harness calls), the final fp32 weights of rank 0, and the lr schedule.
tests/test_ds_harness_cpu.py replays the shim against it without the
reference.

Usage: python tests/golden/make_ds_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DS = "/root/reference/resnet/deepspeed/deepspeed_train.py"
SHIMS = os.path.join(REPO, "distributed_training_amd", "compat", "shims")
OUT = os.path.join(HERE, "ds_harness_ws2.npz")
WS = 2
VARIANTS = [(0, "fp32"), (0, "bf16"), (2, "fp32"), (2, "bf16")]
N_SAMPLES = 288  # three steps of the reference's train_batch_size 96 (48 per rank)


def ds_config(stage: int, dtype: str) -> dict:
    """R:resnet/deepspeed/deepspeed_train.py:172-220, values unchanged."""
    return {
        "train_batch_size": 96,
        "steps_per_print": 2000,
        "optimizer": {"type": "Adam", "params": {"lr": 0.001, "betas": [0.8, 0.999], "eps": 1e-8,
                                                 "weight_decay": 3e-7}},
        "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 0.001,
                                                     "warmup_num_steps": 1000}},
        "gradient_clipping": 1.0,
        "prescale_gradients": False,
        "bf16": {"enabled": dtype == "bf16"},
        "fp16": {"enabled": dtype == "fp16", "fp16_master_weights_and_grads": False, "loss_scale": 0,
                 "loss_scale_window": 500, "hysteresis": 2, "min_loss_scale": 1, "initial_scale_power": 15},
        "wall_clock_breakdown": False,
        "zero_optimization": {"stage": stage, "allgather_partitions": True, "reduce_scatter": True,
                              "allgather_bucket_size": 50000000, "reduce_bucket_size": 50000000,
                              "overlap_comm": True, "contiguous_gradients": True, "cpu_offload": False},
    }


def micro():
    from distributed_training_amd.resnet import BasicBlock, ResNet

    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=4)


def dataset():
    g = torch.Generator().manual_seed(2024)
    return torch.utils.data.TensorDataset(torch.rand(N_SAMPLES, 3, 32, 32, generator=g),
                                          torch.randint(0, 10, (N_SAMPLES,), generator=g))


class RecordingCE(nn.CrossEntropyLoss):
    """The harness's criterion, recording each step's loss."""

    def __init__(self):
        super().__init__()
        self.losses = []

    def forward(self, x, y):
        loss = super().forward(x, y)
        self.losses.append(float(loss.detach().float()))
        return loss


def load_reference():
    spec = importlib.util.spec_from_file_location("ref_deepspeed_train", REF_DS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def worker(rank, ws, port, q):
    sys.path[:0] = [SHIMS, os.path.join(HERE, "_shim"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    import deepspeed

    deepspeed.init_distributed(dist_backend="gloo")  # R:deepspeed_train.py:168 (gloo: CPU)
    ref = load_reference()
    out = {}
    for stage, dtype in VARIANTS:
        sys.argv = ["deepspeed_train.py", "--deepspeed", "--stage", str(stage), "--dtype", dtype]
        args = ref.add_argument()  # R:deepspeed_train.py:27-129, unchanged
        torch.manual_seed(0)
        model = micro()
        parameters = filter(lambda p: p.requires_grad, model.parameters())  # :229
        engine, _, trainloader, sched = deepspeed.initialize(args=args, model=model, model_parameters=parameters,
                                                            training_data=dataset(), config=ds_config(stage, dtype))
        target_dtype = None  # :244-248
        if engine.bfloat16_enabled():
            target_dtype = torch.bfloat16
        elif engine.fp16_enabled():
            target_dtype = torch.half
        crit = RecordingCE()
        lrs = []
        real_step = engine.step

        def step_and_record(*a, **k):
            r = real_step(*a, **k)
            lrs.append(engine.get_lr()[0])
            return r

        engine.step = step_and_record
        ref.train_epoch(0, 1, model, crit, trainloader, "cpu", engine, target_dtype)  # :133-158, unchanged
        key = f"stage{stage}_{dtype}"
        out[f"{key}_losses"] = np.array(crit.losses, dtype=np.float64)
        out[f"{key}_lrs"] = np.array(lrs, dtype=np.float64)
        out[f"{key}_weights"] = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).numpy()
        out[f"{key}_args"] = np.array([args.stage, int(args.deepspeed), args.batch_size, args.epochs])
    q.put((rank, out))


def main():
    sys.path.insert(0, REPO)
    from tests._dist_util import free_port

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, WS, port, q)) for r in range(WS)]
    for p in ps:
        p.start()
    res = dict(q.get() for _ in range(WS))
    for p in ps:
        p.join(600)
    blob = {}
    for rank, out in sorted(res.items()):
        for k, v in out.items():
            if k.endswith("_weights") and rank != 0:
                assert np.array_equal(v, res[0][k]), f"{k}: replicas diverged"
                continue
            blob[f"r{rank}_{k}"] = v
    np.savez_compressed(OUT, **blob)
    print(f"wrote {OUT}: {sorted(blob)}")


if __name__ == "__main__":
    main()
