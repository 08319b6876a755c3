"""Pin the oracle against the golden fixtures made by running the reference's
own train step (R:resnet/pytorch_ddp/ddp_train.py:52-75) under torch DDP +
gloo (tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def n_params(z):
    return len(z["param_names"])


@pytest.mark.parametrize("name", ["ddp_sgd_ws2.npz", "ddp_adam_ws2.npz", "ddp_sgd_ws4.npz"])
def test_oracle_average_matches_reference_ddp(golden_dir, name):
    z = load(golden_dir, name)
    ws = int(z["ws"])
    n = n_params(z)
    local = [[z[f"local/{r}/{i}"] for i in range(n)] for r in range(ws)]
    avg = O.ddp_average(local)
    for i in range(n):
        ref = z[f"grad/0/{i}"]
        if ws <= 2:
            # bitwise at ws in {1, 2} (exact 1/ws prescale, order-free 2-way sum)
            assert np.array_equal(avg[i], ref), f"param {i}"
        else:
            bound = 4 * (ws - 1) * 2.0 ** -24 * sum(np.abs(l[i]) for l in local) / ws
            assert np.all(np.abs(avg[i] - ref) <= bound + 1e-30), f"param {i}"


def test_oracle_padded_layout_is_layout_free(golden_dir):
    z = load(golden_dir, "ddp_sgd_ws2.npz")
    n = n_params(z)
    local = [[z[f"local/{r}/{i}"] for i in range(n)] for r in range(2)]
    a = O.ddp_average(local, align=0)
    b = O.ddp_average(local, align=64)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def _sgd_chain(z, n, steps):
    params = [z[f"init/{i}"].reshape(-1).copy() for i in range(n)]
    bufs = [None] * n
    outs = []
    for s in range(steps):
        for i in range(n):
            g = z[f"grad/{s}/{i}"].reshape(-1)
            p, b = O.sgd(params[i], g, bufs[i], 0.1, 0.9, 0.0, 1e-4, False, False, bufs[i] is None)
            params[i], bufs[i] = p, b
        outs.append([p.copy() for p in params])
    return outs


@pytest.mark.parametrize("name", ["ddp_sgd_ws2.npz", "ddp_sgd_ws4.npz"])
def test_oracle_sgd_reproduces_reference_weights(golden_dir, name):
    z = load(golden_dir, name)
    n = n_params(z)
    outs = _sgd_chain(z, n, int(z["steps"]))
    for s, ps in enumerate(outs):
        for i in range(n):
            ref = z[f"param/{s}/{i}"].reshape(-1)
            # post-step SGD weights rtol 1e-5, atol 1e-7
            np.testing.assert_allclose(ps[i], ref, rtol=1e-5, atol=1e-7, err_msg=f"step {s} param {i}")


def test_oracle_adam_reproduces_reference_weights(golden_dir):
    z = load(golden_dir, "ddp_adam_ws2.npz")
    n = n_params(z)
    ws = int(z["ws"])
    lr = 1e-3 * ws  # R:resnet/pytorch_ddp/ddp_train.py:97,110
    params = [z[f"init/{i}"].reshape(-1).copy() for i in range(n)]
    m = [np.zeros_like(p) for p in params]
    v = [np.zeros_like(p) for p in params]
    for s in range(int(z["steps"])):
        for i in range(n):
            g = z[f"grad/{s}/{i}"].reshape(-1)
            params[i], m[i], v[i] = O.adam(params[i], g, m[i], v[i], s + 1, lr)
            ref = z[f"param/{s}/{i}"].reshape(-1)
            # SURVEY §8c Adam tolerance: atol = lr*1e-3
            assert np.max(np.abs(params[i] - ref)) <= lr * 1e-3, f"step {s} param {i}"


def test_oracle_bf16_compress_hook(golden_dir):
    """torch's bf16_compress_hook: buffer.to(bf16).div_(ws) -> all-reduce -> copy back."""
    z = load(golden_dir, "ddp_bf16hook_ws2.npz")
    n = n_params(z)
    ws = int(z["ws"])
    local = [[z[f"local/{r}/{i}"] for i in range(n)] for r in range(ws)]
    shapes = [l.shape for l in local[0]]
    flats = [O.pack(gs, "bf16", float(ws), 2) for gs in local]
    summed = O.allreduce_sum(flats)
    out = O.unpack(summed, shapes, np.float32, flat_dtype=O.BF16)
    for i in range(n):
        assert np.array_equal(out[i], z[f"grad/0/{i}"]), f"param {i}"


OPT_CASES = {
    "sgd_plain": ("sgd", dict(lr=0.1)),
    "sgd_mom_wd": ("sgd", dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
    "sgd_nesterov": ("sgd", dict(lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-4)),
    "sgd_damp": ("sgd", dict(lr=0.05, momentum=0.8, dampening=0.3)),
    "adam_ref": ("adam", dict(lr=2e-3)),
    "adam_wd": ("adam", dict(lr=1e-3, beta1=0.8, weight_decay=3e-7)),
    "adamw_ds": ("adamw", dict(lr=1e-3, beta1=0.8, weight_decay=3e-7)),
}


@pytest.mark.parametrize("case", list(OPT_CASES))
def test_oracle_optimizers_vs_torch(golden_dir, case):
    z = load(golden_dir, "optim.npz")
    kind, kw = OPT_CASES[case]
    sizes = list(z["sizes"])
    for i in range(len(sizes)):
        p = z[f"{case}/p0/{i}"].copy()
        buf, m, v = None, np.zeros_like(p), np.zeros_like(p)
        for s in range(3):
            g = z[f"{case}/g/{s}/{i}"]
            if kind == "sgd":
                mom = kw.get("momentum", 0.0)
                p, nb = O.sgd(p, g, buf, kw["lr"], mom, kw.get("dampening", 0.0), kw.get("weight_decay", 0.0),
                              kw.get("nesterov", False), False, buf is None)
                buf = nb if mom else None
                np.testing.assert_allclose(p, z[f"{case}/p/{s}/{i}"], rtol=1e-5, atol=1e-7)
            else:
                p, m, v = O.adam(p, g, m, v, s + 1, kw["lr"], kw.get("beta1", 0.9), 0.999, 1e-8,
                                 kw.get("weight_decay", 0.0), kind == "adamw")
                assert np.max(np.abs(p - z[f"{case}/p/{s}/{i}"])) <= kw["lr"] * 1e-3


@pytest.mark.parametrize("case", ["clip_big", "clip_small"])
def test_oracle_clip_vs_torch(golden_dir, case):
    z = load(golden_dir, "optim.npz")
    sizes = list(z["sizes"])
    gs = [z[f"{case}/g/{i}"] for i in range(len(sizes))]
    total = O.sqnorm(gs) ** 0.5
    assert abs(total - float(z[f"{case}/norm"])) <= 1e-5 * total
    coef = np.float32(O.clip_coef(np.float32(total), 1.0))
    for i, g in enumerate(gs):
        np.testing.assert_allclose(g * coef, z[f"{case}/out/{i}"], rtol=2e-6, atol=1e-12)


def test_oracle_bucket_assignment_vs_torch(golden_dir):
    with open(os.path.join(golden_dir, "buckets.json")) as f:
        d = json.load(f)
    for key, v in d.items():
        nbytes = [n * v["element_size"] for n in v["numels"]]
        init = O.bucket_assignment(nbytes, [2**62])
        assert init == v["init_assignment"], key
        rebuilt = O.bucket_assignment(nbytes, [1024 * 1024, 25 * 1024 * 1024], order=v["ready_order"])
        assert rebuilt == v["rebuilt_assignment"], key


def test_rebuilt_bucket_bytes_match_survey(golden_dir):
    """SURVEY §8a A3 lists the rebuilt fp32 bucket sizes; the fixture must agree."""
    with open(os.path.join(golden_dir, "buckets.json")) as f:
        d = json.load(f)
    want = {
        "resnet18/float32": [9461800, 26494976, 8769792],
        "resnet50/float32": [8196000, 31502336, 26255360, 26550272, 9724160],
        "resnet50/bfloat16": [4098000, 28878848, 18137216],
    }
    for key, sizes in want.items():
        v = d[key]
        got = [sum(v["numels"][i] for i in b) * v["element_size"] for b in v["rebuilt_assignment"]]
        assert got == sizes, key
