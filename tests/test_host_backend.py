"""libgsync on the host (no GPU): the C ABI loads and exports every symbol
include/gsync.h declares, its host backend reproduces the oracle bit for bit,
its bucket assignment reproduces torch's, and errors surface as exceptions."""
import json
import os
import re

import numpy as np
import pytest
import torch

from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(REPO, "include", "gsync.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(gs_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    import ctypes

    from distributed_training_amd import _lib as L

    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 40
    for s in syms:
        assert hasattr(lib, s), f"libgsync does not export {s}"
        assert isinstance(getattr(lib, s), ctypes._CFuncPtr)
    assert set(syms) == set(L.SIGNATURES), set(syms) ^ set(L.SIGNATURES)
    assert lib.gs_version() == 1000


def test_hip_request_without_device_fails_loudly():
    from distributed_training_amd import _lib as L
    from distributed_training_amd.multi_tensor import TensorListPlan

    if torch.cuda.is_available():
        pytest.skip("host has a GPU")
    with pytest.raises(L.GsyncError, match="not available"):
        TensorListPlan([4, 5], torch.device("cuda", 0))


def test_invalid_arguments_raise():
    from distributed_training_amd import _lib as L
    from distributed_training_amd.multi_tensor import TensorListPlan

    p = TensorListPlan([4], torch.device("cpu"))
    with pytest.raises(L.GsyncError, match="slot out of range"):
        L.check(L.lib().gs_plan_set_ptrs(p.handle, 9, L.ptr_array([0]), None), "x")
    with pytest.raises(L.GsyncError):
        TensorListPlan([4], torch.device("cpu"), align=3)


RAGGED = [1, 3, 4, 5, 63, 64, 65, 1000, 16385] + [1 + (i % 7) for i in range(40)]


def rand(sizes, seed, scale=1.0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(n, generator=g) * scale).to(dtype) for n in sizes]


def np32(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).reshape(-1)
    return t.numpy().reshape(-1)


@pytest.mark.parametrize("align", [0, 64])
@pytest.mark.parametrize("flat_dt,mode,scale", [(torch.float32, 1, 0.5), (torch.float32, 1, float(np.float32(1 / 3))),
                                                (torch.bfloat16, 1, 0.25), (torch.bfloat16, 2, 3.0),
                                                (torch.float32, 0, 1.0)])
def test_host_pack_unpack_bitwise(align, flat_dt, mode, scale):
    from distributed_training_amd.multi_tensor import TensorListPlan

    ts = rand(RAGGED, 1)
    plan = TensorListPlan([t.numel() for t in ts], torch.device("cpu"), align)
    plan.set_ptrs(1, ts)
    flat = torch.zeros(plan.flat_numel, dtype=flat_dt)
    plan.pack(1, torch.float32, flat, scale, mode)
    ref = O.pack([np32(t) for t in ts], "bf16" if flat_dt == torch.bfloat16 else "f32", scale, mode, align)
    assert np.array_equal(np32(flat), ref)
    outs = [torch.empty_like(t) for t in ts]
    plan.set_ptrs(2, outs)
    plan.unpack(flat, 2, torch.float32)
    back = O.unpack(ref, [t.shape for t in ts], np.float32, align,
                    flat_dtype=O.BF16 if flat_dt == torch.bfloat16 else O.F32)
    for o, r in zip(outs, back):
        assert np.array_equal(np32(o), r.reshape(-1))


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("first,nesterov,damp", [(True, False, 0.0), (False, False, 0.0), (False, True, 0.0),
                                                 (False, False, 0.3)])
def test_host_sgd_bitwise(gdt, first, nesterov, damp):
    from distributed_training_amd.multi_tensor import TensorListPlan

    ps, gs, bs = rand(RAGGED, 2), rand(RAGGED, 3, 0.1, gdt), rand(RAGGED, 4, 0.01)
    ref = [O.sgd(np32(p), np32(g), np32(b), 0.1, 0.9, damp, 1e-4, nesterov, False, first) for p, g, b in zip(ps, gs, bs)]
    plan = TensorListPlan([p.numel() for p in ps], torch.device("cpu"))
    plan.set_ptrs(0, ps)
    plan.set_ptrs(1, gs)
    plan.set_ptrs(2, bs)
    plan.sgd(gdt, 0.1, 0.9, damp, 1e-4, nesterov, False, first)
    for p, b, (rp, rb) in zip(ps, bs, ref):
        assert np.array_equal(np32(p), rp)
        assert np.array_equal(np32(b), rb)


@pytest.mark.parametrize("adamw,wd", [(False, 0.0), (False, 3e-7), (True, 1e-2)])
def test_host_adam_bitwise(adamw, wd):
    from distributed_training_amd.multi_tensor import TensorListPlan

    ps, gs, ms = rand(RAGGED, 5), rand(RAGGED, 6, 0.1), rand(RAGGED, 7, 0.01)
    vs = [v.abs() for v in rand(RAGGED, 8, 1e-4)]
    step, lr, b1, b2, eps = 3, 1e-3, 0.8, 0.999, 1e-8
    ref = [O.adam(np32(p), np32(g), np32(m), np32(v), step, lr, b1, b2, eps, wd, adamw) for p, g, m, v in zip(ps, gs, ms, vs)]
    plan = TensorListPlan([p.numel() for p in ps], torch.device("cpu"))
    for s, ts in enumerate((ps, gs, ms, vs)):
        plan.set_ptrs(s, ts)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    plan.adam(torch.float32, lr, b1, b2, eps, wd, adamw, False, -(lr / bc1), bc2 ** 0.5)
    for p, m, v, (rp, rm, rv) in zip(ps, ms, vs, ref):
        assert np.array_equal(np32(p), rp)
        assert np.array_equal(np32(m), rm)
        assert np.array_equal(np32(v), rv)


def test_fused_optimizers_vs_torch_on_cpu(golden_dir):
    """FusedSGD / FusedAdam (host backend) against torch.optim on the golden
    single-step fixture (SURVEY §8c tolerances)."""
    from distributed_training_amd.optim import FusedAdam, FusedAdamW, FusedSGD

    z = np.load(os.path.join(golden_dir, "optim.npz"), allow_pickle=False)
    sizes = list(z["sizes"])
    for case, cls, kw in (("sgd_mom_wd", FusedSGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
                          ("sgd_nesterov", FusedSGD, dict(lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-4)),
                          ("adam_ref", FusedAdam, dict(lr=2e-3)),
                          ("adamw_ds", FusedAdamW, dict(lr=1e-3, betas=(0.8, 0.999), eps=1e-8, weight_decay=3e-7))):
        params = [torch.nn.Parameter(torch.from_numpy(z[f"{case}/p0/{i}"].copy())) for i in range(len(sizes))]
        opt = cls(params, **kw)
        for s in range(3):
            for i, p in enumerate(params):
                p.grad = torch.from_numpy(z[f"{case}/g/{s}/{i}"].copy())
            opt.step()
            for i, p in enumerate(params):
                ref = z[f"{case}/p/{s}/{i}"]
                if cls is FusedSGD:
                    np.testing.assert_allclose(p.detach().numpy(), ref, rtol=1e-5, atol=1e-7)
                else:
                    assert np.max(np.abs(p.detach().numpy() - ref)) <= kw["lr"] * 1e-3
        # torch-compatible state_dict round trip
        sd = opt.state_dict()
        opt2 = cls(params, **kw)
        opt2.load_state_dict(sd)
        key = "momentum_buffer" if cls is FusedSGD else "exp_avg"
        assert key in opt2.state[params[0]]


def test_cpp_bucket_assignment_vs_torch(golden_dir):
    from distributed_training_amd.ddp import compute_bucket_assignment_by_size

    with open(os.path.join(golden_dir, "buckets.json")) as f:
        d = json.load(f)
    for key, v in d.items():
        dt = torch.float32 if v["element_size"] == 4 else torch.bfloat16
        ts = [torch.empty(n, dtype=dt, device="meta") for n in v["numels"]]
        assert compute_bucket_assignment_by_size(ts, [2**62]) == v["init_assignment"], key
        got = compute_bucket_assignment_by_size(ts, [1024 * 1024, 25 * 1024 * 1024], order=v["ready_order"])
        assert got == v["rebuilt_assignment"], key


def test_clip_grad_norm_cpu(golden_dir):
    from distributed_training_amd.optim import clip_grad_norm_

    z = np.load(os.path.join(golden_dir, "optim.npz"), allow_pickle=False)
    sizes = list(z["sizes"])
    for case in ("clip_big", "clip_small"):
        params = [torch.nn.Parameter(torch.zeros(int(n))) for n in sizes]
        for i, p in enumerate(params):
            p.grad = torch.from_numpy(z[f"{case}/g/{i}"].copy())
        norm = clip_grad_norm_(params, 1.0)
        assert abs(norm.item() - float(z[f"{case}/norm"])) <= 1e-5 * float(z[f"{case}/norm"])
        for i, p in enumerate(params):
            np.testing.assert_allclose(p.grad.numpy(), z[f"{case}/out/{i}"], rtol=2e-6, atol=1e-12)


def test_state_dict_keys_layout(golden_dir):
    """Checkpoint layout: torchvision ResNet keys under DDP's `module.` prefix."""
    from distributed_training_amd.resnet import resnet18, resnet50

    with open(os.path.join(golden_dir, "state_dict_keys.json")) as f:
        keys = json.load(f)
    assert ["module." + k for k in resnet50().state_dict().keys()] == keys["resnet50"]
    assert ["module." + k for k in resnet18(num_classes=10).state_dict().keys()] == keys["resnet18"]
    # torchvision-0.15 names (spot checks)
    for k in ("module.conv1.weight", "module.bn1.running_mean", "module.layer1.0.downsample.0.weight",
              "module.layer4.2.bn3.num_batches_tracked", "module.fc.bias"):
        assert k in keys["resnet50"]


def _host_bucketer(numels, buckets, flags=0, div=2.0, align=64):
    import ctypes

    from distributed_training_amd import _lib as L

    h = ctypes.c_void_p()
    counts = [len(b) for b in buckets]
    members = [i for b in buckets for i in b]
    L.check(L.lib().gs_bucketer_create(None, L.GS_DEV_HOST, 0, len(numels), L.i64_array(numels), L.GS_F32,
                                       len(buckets), L.i32_array(counts), L.i32_array(members), L.GS_F32, align,
                                       div, flags, ctypes.byref(h)), "create")
    bufs = []
    for b in range(len(buckets)):
        n = ctypes.c_int64()
        L.check(L.lib().gs_bucketer_bucket_numel(h, b, ctypes.byref(n)), "numel")
        bufs.append(torch.zeros(n.value))
        L.check(L.lib().gs_bucketer_set_bucket_buffer(h, b, bufs[-1].data_ptr()), "set")
    return h, bufs


def test_bucketer_protocol_and_order():
    """Reducer semantics: buckets launch strictly in index order, a parameter is
    marked once per backward, finalize needs every bucket (torch's messages)."""
    import ctypes

    from distributed_training_amd import _lib as L

    lib = L.lib()
    grads = [torch.full((n,), float(i + 1)) for i, n in enumerate([5, 70, 3, 130])]
    h, bufs = _host_bucketer([g.numel() for g in grads], [[3, 2], [1, 0]])
    ready = (ctypes.c_int32 * 4)()
    nr = ctypes.c_int32()
    with pytest.raises(L.GsyncError, match="prepare"):
        L.check(lib.gs_bucketer_mark_ready(h, 0, grads[0].data_ptr(), None, ready, ctypes.byref(nr)), "mark")
    L.check(lib.gs_bucketer_prepare(h, None), "prepare")
    # bucket 1 completes first but must wait for bucket 0
    for p in (1, 0):
        L.check(lib.gs_bucketer_mark_ready(h, p, grads[p].data_ptr(), None, ready, ctypes.byref(nr)), "mark")
        assert nr.value == 0
    with pytest.raises(L.GsyncError, match="only once"):
        L.check(lib.gs_bucketer_mark_ready(h, 0, grads[0].data_ptr(), None, ready, ctypes.byref(nr)), "mark")
    with pytest.raises(L.GsyncError, match="finished reduction"):
        L.check(lib.gs_bucketer_finalize(h, None), "finalize")
    L.check(lib.gs_bucketer_mark_ready(h, 3, grads[3].data_ptr(), None, ready, ctypes.byref(nr)), "mark")
    assert nr.value == 0
    L.check(lib.gs_bucketer_mark_ready(h, 2, grads[2].data_ptr(), None, ready, ctypes.byref(nr)), "mark")
    assert [ready[k] for k in range(nr.value)] == [0, 1]
    # packed with the 1/ws prescale at 64-element aligned offsets
    assert torch.equal(bufs[0][:130], torch.full((130,), 4.0 * 0.5))
    assert torch.equal(bufs[0][130:192], torch.zeros(62))
    assert torch.equal(bufs[0][192:195], torch.full((3,), 3.0 * 0.5))
    for b in bufs:
        b.mul_(2.0)  # stand-in for the SUM all-reduce of two identical ranks
    L.check(lib.gs_bucketer_finalize(h, None), "finalize")
    for i, g in enumerate(grads):
        assert torch.equal(g, torch.full_like(g, float(i + 1)))
    L.check(lib.gs_bucketer_destroy(h), "destroy")


def test_bucketer_mark_unused_packs_zeros():
    import ctypes

    from distributed_training_amd import _lib as L

    lib = L.lib()
    g0 = torch.ones(10)
    h, bufs = _host_bucketer([10, 20], [[1, 0]])
    bufs[0].fill_(7.0)
    ready = (ctypes.c_int32 * 2)()
    nr = ctypes.c_int32()
    L.check(lib.gs_bucketer_prepare(h, None), "prepare")
    L.check(lib.gs_bucketer_mark_ready(h, 0, g0.data_ptr(), None, ready, ctypes.byref(nr)), "mark")
    L.check(lib.gs_bucketer_mark_unused(h, None, ready, ctypes.byref(nr)), "unused")
    assert nr.value == 1
    assert torch.equal(bufs[0][:20], torch.zeros(20))  # the unused parameter's slot
    L.check(lib.gs_bucketer_finalize(h, None), "finalize")
    L.check(lib.gs_bucketer_destroy(h), "destroy")


def test_plan_task_sizing():
    """Balanced decomposition: ~1920 tasks (one resident wave of <= 2048 workgroups),
    whole 256-unit iterations, clamped to [256, 4096] units (1 unit = 4 elements)."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.multi_tensor import TensorListPlan
    from distributed_training_amd.resnet import MODELS

    cpu = torch.device("cpu")
    small = TensorListPlan([10, 1000], cpu)
    assert small.task_units == 256 and small.n_tasks == 1
    for name in ("resnet18", "resnet50", "resnet152"):
        sizes = [p.numel() for p in MODELS[name]().parameters()]
        plan = TensorListPlan(sizes, cpu)
        units = sum((n + 3) // 4 for n in sizes)
        assert plan.task_units % 256 == 0 and 256 <= plan.task_units <= 4096
        assert name == "resnet152" or plan.n_tasks <= 2048, (name, plan.n_tasks)
        assert plan.n_tasks >= units // plan.task_units
    huge = TensorListPlan([400_000_000], cpu)
    assert huge.task_units == 4096
    with pytest.raises(L.GsyncError, match="host plans"):
        small.timer_enable(4)


def test_host_threads_bitwise():
    """The host backend's threaded loops (gs_set_host_threads) give the same bits
    as one thread: every op is elementwise, the split only changes who computes."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.multi_tensor import TensorListPlan

    sizes = [1_000_003, 7, 300_000, 65_536 * 3 + 5]
    g = torch.Generator().manual_seed(0)

    def run(threads):
        torch.manual_seed(0)
        ps = [torch.randn(n, generator=torch.Generator().manual_seed(i)) for i, n in enumerate(sizes)]
        gs = [torch.randn(n, generator=torch.Generator().manual_seed(10 + i)) * 0.01 for i, n in enumerate(sizes)]
        ms = [torch.zeros(n) for n in sizes]
        vs = [torch.zeros(n) for n in sizes]
        plan = TensorListPlan(sizes, torch.device("cpu"), align=64)
        for k, ts in enumerate((ps, gs, ms, vs)):
            plan.set_ptrs(k, ts)
        flat = torch.zeros(plan.flat_numel, dtype=torch.bfloat16)
        old = torch.get_num_threads()
        torch.set_num_threads(threads)  # the Python layer forwards it to the library
        try:
            plan.pack(1, torch.float32, flat, 0.25, L.GS_SCALE_MUL)
            plan.adam(torch.float32, 1e-3, 0.9, 0.999, 1e-8, 1e-2, True, False, -1e-3, 0.7)
            found = torch.zeros(1)
            plan.unscale_check(1, torch.float32, torch.tensor([0.5]), found)
        finally:
            torch.set_num_threads(old)
        return [flat.clone()] + ps + ms + vs + gs + [found]

    a, b = run(1), run(8)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
