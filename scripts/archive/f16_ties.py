"""fp32 -> fp16 rounding of exact ties (value = (2k+1)/2 fp16 ulps) on the
GPU: libgsync's pack kernel (fp16 bucket), torch's .half(), against numpy's
IEEE round-to-nearest-even.  Prints the mismatch counts per path."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402

rng = np.random.default_rng(0)
n = 1 << 16
# random fp16 values, then + half an ulp: every value is an exact tie in fp16
h = rng.standard_normal(n).astype(np.float16)
h = h[np.isfinite(h) & (np.abs(h) > 6.2e-5)]
up = np.nextafter(h, np.float16(np.inf) * np.sign(h)).astype(np.float16)
ties = ((h.astype(np.float64) + up.astype(np.float64)) / 2).astype(np.float32)
assert np.all(ties.astype(np.float64) == (h.astype(np.float64) + up.astype(np.float64)) / 2)
want = ties.astype(np.float16)  # numpy: IEEE round-to-nearest-even
dev = torch.device("cuda", 0)
x = torch.from_numpy(ties).to(dev)
t_half = x.half().cpu().numpy()
plan = TensorListPlan([x.numel()], dev, align=64)
plan.set_ptrs(1, [x])
flat = torch.zeros(plan.flat_numel, device=dev, dtype=torch.float16)
plan.pack(1, torch.float32, flat, 1.0, 0)
g_pack = flat[: x.numel()].cpu().numpy()
print("ties", len(ties))
print("torch .half() != RNE:", int((t_half.view(np.uint16) != want.view(np.uint16)).sum()))
print("libgsync pack  != RNE:", int((g_pack.view(np.uint16) != want.view(np.uint16)).sum()))
bad = np.nonzero(g_pack.view(np.uint16) != want.view(np.uint16))[0][:4]
print([(float(ties[i]), float(g_pack[i]), float(want[i])) for i in bad])

# the fused update's low-precision param write (ZeRO fp16 / bf16 models): step size 0 keeps
# p_new == p exactly, so the fp16 copy must be RNE(p)
from distributed_training_amd.multi_tensor import update_task_units  # noqa: E402

for kind in ("adam", "sgd"):
    up = TensorListPlan([x.numel()], dev, task_units=update_task_units(dev))
    p = x.clone()
    gr = torch.full_like(x, 1e-3)
    m = torch.zeros_like(x)
    v = torch.zeros_like(x)
    p16 = torch.zeros(x.numel(), device=dev, dtype=torch.float16)
    up.set_ptrs(0, [p]); up.set_ptrs(1, [gr]); up.set_ptrs(2, [m])
    if kind == "adam":
        up.set_ptrs(3, [v]); up.set_ptrs(4, [p16])
        up.adam(torch.float32, 0.0, 0.9, 0.999, 1e-8, 0.0, True, False, -0.0, 1.0, lowp_dtype=torch.float16)
    else:
        up.set_ptrs(3, [p16])
        up.sgd(torch.float32, 0.0, 0.9, 0.0, 0.0, False, False, True, lowp_dtype=torch.float16)
    torch.cuda.synchronize()
    same_p = torch.equal(p, x)
    got = p16.cpu().numpy()
    print(kind, "p unchanged:", same_p, " lowp != RNE:", int((got.view(np.uint16) != want.view(np.uint16)).sum()))
    bad = np.nonzero(got.view(np.uint16) != want.view(np.uint16))[0][:4]
    print([(float(ties[i]), float(got[i]), float(want[i])) for i in bad])
