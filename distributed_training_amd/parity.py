"""Cross-rank self-check of one synchronising step (the driver's N > 1 runs
must tell a correct gradient sync from a wrong one).

After ``bench.py``'s timed region every rank runs ONE more step with the local
gradients of a few parameters captured in the autograd hooks (before the
bucket pack), then checks, through the engine's own communicator (libgsync's
RCCL communicator on an nccl group; the gloo group otherwise):

* averaged gradients == Σ_r g_r · float(1/ws), the Reducer's arithmetic
  (T:include/torch/csrc/distributed/c10d/reducer.hpp:275 mul_out by 1/div_factor,
  then the SUM all-reduce): the local grads are all-gathered and the expected
  value is formed in rank order in fp32.  Bitwise at ws ≤ 2 (scaling by 1/2 is
  exact and a 2-term sum is order-free); at ws > 2 within SURVEY.md §8c's
  |Δ| ≤ 4(n−1)·2⁻²⁴·Σ_r|g_r|/n (RCCL's reduction order is not rank order);
  low-precision buckets within 2⁻⁷·max|g| per tensor.
  ZeRO-2: the reduce-scattered shards are all-gathered first.
* post-step parameters identical on every rank: per-tensor checksums (Σ of the
  tensor's 32-bit words as int64, Σ of its values in fp64) all-reduced MIN and
  MAX — equal iff every rank holds the same bits (up to checksum collisions);
* module buffers identical after the per-forward broadcast
  (T:nn/parallel/distributed.py:2178-2221; DDP only: ZeRO broadcasts once).

Reference behaviour checked: R:resnet/pytorch_ddp/ddp_train.py:84,95,109-114
(NCCL DDP at world size 2) and R:resnet/deepspeed/deepspeed_train.py:210-219
(ZeRO reduce-scatter + all-gather).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib as L


class _Coll:
    """The engine's communicator for the checks: libgsync RCCL when present,
    else the process group (gloo: CPU copies)."""

    def __init__(self, comm, pg, device):
        self.comm = comm
        self.pg = pg if pg is not None else dist.group.WORLD
        self.device = device
        self.world = dist.get_world_size(self.pg)
        self.backend = "rccl(libgsync)" if comm is not None else dist.get_backend(self.pg)

    def _host(self):
        return self.comm is None and dist.get_backend(self.pg) == "gloo"

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, numel] of every rank's 1-D tensor t."""
        t = t.contiguous().reshape(-1)
        if self.comm is not None:
            out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
            # the checker does not lean on the collective's stream ordering
            torch.cuda.current_stream(t.device).synchronize()
            self.comm.all_gather(t, out, stream=L.stream_ptr(t.device))
            torch.cuda.current_stream(t.device).synchronize()
            return out.view(self.world, -1)
        src = t.cpu() if self._host() else t
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.pg)
        return torch.stack(parts).to(t.device)

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        t = t.clone()
        if self.comm is not None:
            self.comm.all_reduce(t, op=op, stream=L.stream_ptr(t.device))
            torch.cuda.current_stream(t.device).synchronize()
            return t
        src = t.cpu() if self._host() else t
        dist.all_reduce(src, op={"min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX,
                                 "sum": dist.ReduceOp.SUM}[op], group=self.pg)
        return src.to(t.device)


def pick_params(n: int, k: int = 6) -> list[int]:
    """k parameter indices spread over the model (first, last, evenly between)."""
    if n <= k:
        return list(range(n))
    return sorted({round(i * (n - 1) / (k - 1)) for i in range(k)})


def expected_average(local: torch.Tensor, world: int, bucket_dtype: torch.dtype) -> torch.Tensor:
    """Σ_r cast(g_r · float(1/ws)) in rank order, fp32 accumulation
    (local = [world, numel] gathered local grads)."""
    inv = torch.tensor(1.0 / world, dtype=torch.float32)  # float(1.0/div_factor)
    acc = None
    for r in range(world):
        term = (local[r].float() * inv.to(local.device)).to(bucket_dtype).float()
        acc = term if acc is None else acc + term
    return acc


def compare_average(avg: torch.Tensor, local: torch.Tensor, world: int, bucket_dtype: torch.dtype) -> dict:
    exp = expected_average(local, world, bucket_dtype)
    got = avg.float().reshape(-1)
    err = (got - exp).abs()
    if bucket_dtype == torch.float32:
        tol = 4 * (world - 1) * 2.0 ** -24 * local.float().abs().sum(0) / world
        rule = "4(n-1)*2^-24*sum_r|g_r|/n (SURVEY 8c); bitwise required at n<=2"
    else:
        tol = torch.full_like(exp, 2.0 ** -7 * float(local.float().abs().max()))
        rule = "2^-7*max|g| (low-precision buckets, SURVEY 8c)"
    bitwise = bool(torch.equal(got, exp))
    ratio = float((err / tol.clamp_min(1e-38)).max()) if err.numel() else 0.0
    within = bool((err <= tol).all())
    ok = bitwise if (world <= 2 and bucket_dtype == torch.float32) else within
    return {"elements": int(got.numel()), "bitwise_equal": bitwise, "max_abs_err": float(err.max()) if err.numel() else 0.0,
            "max_err_over_tol": ratio, "tolerance": rule, "ok": ok}


def tensor_checksums(tensors) -> torch.Tensor:
    """[2 * len] int64: per tensor, Σ of its 32-bit words and Σ of its values
    (fp64, bit-cast to int64) — identical bits give identical checksums."""
    out = []
    for t in tensors:
        t = t.detach().contiguous()
        flat = t.reshape(-1)
        if flat.numel() == 0:
            out += [torch.zeros((), dtype=torch.int64, device=t.device)] * 2
            continue
        if flat.element_size() == 2:
            words = flat.view(torch.int16).to(torch.int64)
        elif flat.element_size() == 1:
            words = flat.view(torch.uint8).to(torch.int64)
        else:
            words = flat.view(torch.int32).to(torch.int64)
        out.append(words.sum())
        out.append(flat.double().sum().view(torch.int64) if flat.is_floating_point()
                   else flat.to(torch.int64).sum())
    return torch.stack(out) if out else torch.zeros(0, dtype=torch.int64)


def identical_across_ranks(coll: _Coll, tensors) -> bool:
    cs = tensor_checksums(tensors)
    if cs.numel() == 0:
        return True
    lo = coll.all_reduce(cs, "min")
    hi = coll.all_reduce(cs, "max")
    return bool(torch.equal(lo, hi))


def ddp_parity_step(ddp, optimizer, run_forward_backward, k: int = 6) -> dict:
    """One step of a libgsync DDP engine with the checks above.
    run_forward_backward() does forward + loss.backward() on this rank's batch."""
    params = ddp._params
    idx = pick_params(len(params), k)
    coll = _Coll(ddp._comm, ddp.process_group, ddp.device)
    ddp._capture_local = {i: None for i in idx}
    try:
        run_forward_backward()
    finally:
        cap = ddp._capture_local
        ddp._capture_local = None
    torch.cuda.synchronize(ddp.device) if ddp.device.type == "cuda" else None
    # compare per bucket dtype (a model with params of several dtypes has buckets of each)
    bucket_of = {i: b for b, members in enumerate(ddp._bucketer.buckets) for i in members}
    by_dt: dict = {}
    for i in idx:
        by_dt.setdefault(ddp._bucketer.bucket_dtypes[bucket_of[i]], []).append(i)
    parts = []
    for dt, ids in by_dt.items():
        local = torch.cat([cap[i].reshape(-1).float() for i in ids])
        avg = torch.cat([params[i].grad.detach().reshape(-1).float() for i in ids])
        parts.append(compare_average(avg, coll.all_gather(local), coll.world, dt))
    grads = parts[0] if len(parts) == 1 else {
        "elements": sum(p["elements"] for p in parts), "bitwise_equal": all(p["bitwise_equal"] for p in parts),
        "max_abs_err": max(p["max_abs_err"] for p in parts),
        "max_err_over_tol": max(p["max_err_over_tol"] for p in parts),
        "tolerance": "; ".join(sorted({p["tolerance"] for p in parts})), "ok": all(p["ok"] for p in parts)}
    grads["checked_params"] = idx
    optimizer.step()
    optimizer.zero_grad(set_to_none=True)
    ddp._sync_buffers()  # what the next forward does first
    if ddp.device.type == "cuda":
        torch.cuda.synchronize(ddp.device)
    w_ok = identical_across_ranks(coll, [p.detach() for p in params])
    b_ok = identical_across_ranks(coll, list(ddp.module.buffers())) if ddp.broadcast_buffers else None
    return {"engine": "ddp", "collective": coll.backend, "world": coll.world, "averaged_grads": grads,
            "weights_identical": w_ok, "buffers_identical": b_ok,
            "ok": bool(grads["ok"] and w_ok and b_ok is not False)}


def zero_parity_step(zero, run_forward_backward, k: int = 6) -> dict:
    """One step of a ZeroDataParallel engine with the checks above."""
    params = zero.params
    idx = pick_params(len(params), k)
    coll = _Coll(zero._comm, zero.pg, zero.device)
    zero._capture_local = {i: None for i in idx}
    try:
        zero.prepare_backward()
        run_forward_backward()
    finally:
        cap = zero._capture_local
        zero._capture_local = None
    if zero.device.type == "cuda":
        torch.cuda.synchronize(zero.device)
    # averaged grads: all-gather the shards (stage 2) or read the bucket (stage 1)
    fulls = []
    for b, shard in enumerate(zero.grad_shards):
        if zero.stage == 2:
            fulls.append(coll.all_gather(shard).reshape(-1))
        else:
            fulls.append(zero.grad_bufs[b])
    avg_parts, loc_parts = [], []
    for i in idx:
        b, off = zero.loc[i]
        p = params[i]
        # the bucket holds each grad in its parameter's memory order (channels_last
        # convs included): view the slot with the parameter's strides, as the
        # engine's own param views are built (zero._build_flat_state)
        avg_parts.append(fulls[b].as_strided(p.size(), p.stride(), off).reshape(-1).float())
        loc_parts.append(cap[i].reshape(-1).float())
    gathered = coll.all_gather(torch.cat(loc_parts))
    grads = compare_average(torch.cat(avg_parts), gathered, coll.world, zero.dtype)
    grads["checked_params"] = idx
    zero.step()
    zero.zero_grad()
    if zero.device.type == "cuda":
        torch.cuda.synchronize(zero.device)
    w_ok = identical_across_ranks(coll, list(zero.param_flats))
    return {"engine": f"zero{zero.stage}", "collective": coll.backend, "world": coll.world,
            "averaged_grads": grads, "weights_identical": w_ok, "buffers_identical": None,
            "ok": bool(grads["ok"] and w_ok)}
