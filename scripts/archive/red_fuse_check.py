"""Checks the in-kernel (two-level ticket) reduction combine against the
combine_partials launch: run once with GS_RED_FUSE=1 and once with 0.
Per case: 20 back-to-back launches give identical bits (counters re-armed,
deterministic order), Σg² within 1e-5 (relative) of an fp64 sum, accumulate
mode adds, the max-kind reduction (unscale check) flags a planted inf, and a
sum (Σx) matches fp64.  Prints one JSON line per case with the values' bits so
that the fused / unfused runs can be diffed."""
import json
import os
import struct
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
r50 = [p.numel() for p in MODELS["resnet50"]().parameters()]
cases = {
    "one": [1],
    "tiny": [5, 7, 3],
    "ragged": [100, 70001, 4096, 1, 1023, 1025],
    "grid_lt_8": [4096 * 3],
    "r50": r50,
    "r50x3": r50 * 3,
}
fuse = os.environ.get("GS_RED_FUSE", "unset")
bad = 0
for name, numels in cases.items():
    g = torch.Generator(device=dev).manual_seed(11)
    xs = [torch.randn(n, device=dev, generator=g) * 0.01 for n in numels]
    plan = TensorListPlan(numels, dev, align=64)
    plan.set_ptrs(1, xs)
    out = torch.zeros(20, device=dev)
    for i in range(20):
        plan.sqnorm(1, torch.float32, out[i:i + 1])
    torch.cuda.synchronize()
    vals = out.tolist()
    same = all(struct.pack("f", v) == struct.pack("f", vals[0]) for v in vals)
    want = sum(float((x.double() ** 2).sum()) for x in xs)
    rel = abs(vals[0] - want) / want
    acc = torch.full((1,), 2.0, device=dev)
    plan.sqnorm(1, torch.float32, acc, accumulate=True)
    s = torch.zeros(1, device=dev)
    plan.sum(1, torch.float32, s)
    want_s = sum(float(x.double().sum()) for x in xs)
    found = torch.zeros(1, device=dev)
    plan.unscale_check(1, torch.float32, None, found)
    clean = float(found.item())
    xs[len(xs) // 2].view(-1)[-1] = float("inf")
    plan.unscale_check(1, torch.float32, None, found)
    flagged = float(found.item())
    xs[len(xs) // 2].view(-1)[-1] = 0.0
    torch.cuda.synchronize()
    ok = (same and rel < 1e-5 and abs(acc.item() - (2.0 + vals[0])) <= 1e-6 * (2.0 + vals[0])
          and abs(s.item() - want_s) <= 1e-5 * sum(float(x.double().abs().sum()) for x in xs)
          and clean == 0.0 and flagged == 1.0)
    bad += not ok
    print(json.dumps({"case": name, "fuse": fuse, "n": sum(numels), "ok": ok, "repeat_bitwise": same,
                      "sqnorm_bits": struct.unpack("I", struct.pack("f", vals[0]))[0], "rel_err": rel,
                      "sum": s.item(), "inf_clean": clean, "inf_flagged": flagged}), flush=True)
# stress: 400 launches of the R50 Σg² while a second stream keeps copying 256 MB
# (uneven load on the CUs the arrivals and the group leaders run on); every
# result must carry the first one's bits
g = torch.Generator(device=dev).manual_seed(5)
xs = [torch.randn(n, device=dev, generator=g) * 0.01 for n in r50]
plan = TensorListPlan(r50, dev, align=64)
plan.set_ptrs(1, xs)
out = torch.zeros(400, device=dev)
src = torch.randn(64 * 2**20, device=dev)
dst = torch.empty_like(src)
side = torch.cuda.Stream(dev)
with torch.cuda.stream(side):
    for _ in range(40):
        dst.copy_(src)
for i in range(400):
    plan.sqnorm(1, torch.float32, out[i:i + 1])
torch.cuda.synchronize()
bits = out.view(torch.int32)
n_diff = int((bits != bits[0]).sum())
bad += n_diff != 0
print(json.dumps({"case": "stress_r50_400_launches_beside_copies", "fuse": fuse, "ok": n_diff == 0,
                  "differing_results": n_diff, "sqnorm_bits": int(bits[0])}), flush=True)
sys.exit(1 if bad else 0)
