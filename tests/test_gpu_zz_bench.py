"""bench.py's output contract on the GPU, at a small size (ResNet-18, 16 images).

* N=1: one JSON line on stdout with the driver's keys, a `roofline` object for
  the fused update kernel and a `grad_sync` object; the process exits 0.
* N=2 through `torch.distributed.run` exactly as the driver launches it, with
  `--pg-backend gloo` (RCCL refuses two ranks on one GPU): barriers, the MAX
  over ranks and the rank-0-only line — the control flow of the driver's
  N = 2/4/8 runs, not a measurement.

The benches run as child processes (never exec'd from this process); the
module is named to run after the other GPU modules."""
import json
import os
import socket
import signal
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--model", "resnet18", "--batch", "16", "--steps", "3", "--warmup", "2", "--cpu-baseline", "0"]
NO_LEGS = ["--zero-leg", "0", "--colossal-leg", "0"]  # configs[3] / [4] legs: on by default


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    """A clean rendezvous for the child: earlier test modules leave this
    process's own MASTER_PORT / RANK / WORLD_SIZE in os.environ (and the port
    still bound by their process group)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("MASTER_PORT", "RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    env["MASTER_PORT"] = str(_port())
    return env


class _Result:
    def __init__(self, returncode, stdout, stderr):
        self.returncode, self.stdout, self.stderr = returncode, stdout, stderr


# Every bench child runs under CHILD_LIMIT_S, below the GPU box's 180 s silence
# window, so a hang fails its test with the child's stderr (and, for the
# multi-rank runs, every rank's stacks) instead of the box killing the suite.
CHILD_LIMIT_S = 170
_CAPMAN = [None]


@pytest.fixture(autouse=True)
def _capture_manager(request):
    _CAPMAN[0] = request.config.pluginmanager.getplugin("capturemanager")
    yield
    _CAPMAN[0] = None


def _heartbeat(msg):
    """One line on the REAL stderr, past pytest's capture: the driver's quiet
    `pytest -q -m gpu` then shows a long bench child making progress."""
    import contextlib

    cm = _CAPMAN[0]
    ctx = cm.global_and_fixture_disabled() if cm is not None else contextlib.nullcontext()
    with ctx:
        sys.stderr.write(msg + "\n")
        sys.stderr.flush()


def _run(cmd, env, timeout=CHILD_LIMIT_S):
    """Run a bench child; its stdout and stderr (the "[bench] ..." progress lines
    and the ranks' logs) go to files under $GSYNC_TEST_PROGRESS_DIR (default
    gpurun_out/test_progress in the repo, which a gpurun box returns).  While it
    runs, every time its stderr file grows a heartbeat line with the newest
    output goes to the real stderr (above), so the test is never silent while
    its child works; a child past `timeout` (< 180 s) is killed with its whole
    session (torchrun and its ranks) and the test fails with its stderr tail."""
    import time

    d = os.environ.get("GSYNC_TEST_PROGRESS_DIR") or os.path.join(REPO, "gpurun_out", "test_progress")
    os.makedirs(d, exist_ok=True)
    name = os.environ.get("PYTEST_CURRENT_TEST", "bench").split(" ")[0].replace("/", "_").replace("::", "__")
    path = os.path.join(d, f"{name}.{os.getpid()}.err")
    opath = path[:-4] + ".out"
    t0 = time.time()
    with open(path, "w") as err, open(opath, "w") as out_f:
        # own session: on a timeout the whole group (torchrun and its ranks) is killed, not only the launcher
        p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=out_f, stderr=err, text=True, start_new_session=True)
        seen = 0
        while True:
            try:
                p.wait(timeout=10)
                break
            except subprocess.TimeoutExpired:
                pass
            size = os.path.getsize(path)
            if size > seen:
                with open(path, errors="replace") as f:
                    f.seek(max(seen, size - 400))
                    tail = [ln for ln in f.read().splitlines() if ln.strip()]
                seen = size
                _heartbeat(f"[{name}] {time.time() - t0:.0f} s: {tail[-1][:200] if tail else ''}")
            if time.time() - t0 > timeout:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                with open(path, errors="replace") as f:
                    raise AssertionError(f"bench child exceeded {timeout} s; stderr tail:\n{f.read()[-6000:]}")
    with open(path, errors="replace") as f:
        stderr = f.read()
    with open(opath) as f:
        stdout = f.read()
    return _Result(p.returncode, stdout, stderr)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check_line(d, n):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "grad_sync"):
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == 3 and d["warmup"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    # the reference's own GPU path (torch DDP + torch.optim.SGD foreach) timed in the same run, at every N
    t = d.get("torch_ddp")
    assert t is not None or "torch_ddp" in d.get("leg_errors", {}), d.get("leg_errors")
    if t is not None:
        assert t["images_per_sec"] > 0 and t["steps"] > 0 and d["vs_baseline_basis"]
        assert abs(d["vs_baseline"] - d["value"] / t["images_per_sec"]) <= 1e-9 * d["vs_baseline"]
    else:
        assert d["vs_baseline"] is None
    assert d["config"]["workload"] and d["config"]["parallelism"] == f"dp{n}"
    assert d["config"]["global_batch"] == 16 * n
    # value = all ranks' images / the (max-over-ranks) timed region
    assert abs(d["value"] - n * 16 * 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["achieved"] > 0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    # the headline is the update beyond the Infinity Cache (true HBM); the timed steps' own
    # launches are the in-step figure beside it, flagged when the cache lifted them
    ins = r["in_step"]
    assert ins["algorithmic_bytes_per_launch"] == 20 * d["config"]["params"]
    assert ins["launches"] == 3 and ins["achieved"] > 0 and isinstance(ins["ic_assisted"], bool)
    assert ins["ic_assisted"] == (ins["achieved"] > r["copy_ceiling"])
    g = d["grad_sync"]
    assert g["n_buckets"] == len(g["bucket_bytes"]) >= 1
    assert g["grad_bytes_per_step"] == 4 * d["config"]["params"]
    # every grad-sync kernel alone on the model's params (the north star's >= 70 % covers them all)
    k = d["grad_sync_kernels"]
    assert set(k["kernels"]) == {"pack_f32", "pack_f32_to_bf16", "unpack_f32", "unpack_f32+sqnorm", "sqnorm_f32",
                                 "sqnorm_f32_after_unpack", "sqnorm_f32_after_unpack_nt",
                                 "pack_bf16", "unpack_bf16_to_f32", "sgd_momentum_wd", "sqnorm_partial_f32",
                                 "clip_path_sgd", "adam", "clip_grad_norm"}
    # the folded clip path: Σg² partials + the clipped update, both launches in one row
    assert k["kernels"]["clip_path_sgd"]["alg_bytes"] == 24 * d["config"]["params"]
    assert k["kernels"]["clip_path_sgd"]["avg_ms"] > k["kernels"]["sgd_momentum_wd"]["avg_ms"]
    assert all(r["GBps"] > 0 and abs(r["frac"] - r["GBps"] / 8000.0) < 1e-12 for r in k["kernels"].values())
    assert k["params"] == d["config"]["params"]
    # the same rows on a > 256 MiB working set (true HBM), and the headline kernel's rate there
    b = k["beyond_ic"]
    assert set(b["kernels"]) == set(k["kernels"]) and b["params"] > 100_000_000
    assert r["frac"] == r["frac_beyond_ic"] == b["kernels"]["sgd_momentum_wd"]["frac"]
    assert r["algorithmic_bytes_per_launch"] == 20 * b["params"] and r["launches"] == k["iters"]
    assert r["frac_of_copy_ceiling"] <= 1.1  # a true-HBM figure: not above the copy ceiling (box spread aside)
    # ... read against a plain float4 stream of the same 3R2W mix (committed probe run)
    assert r["plain_stream_ceiling"]["case"].startswith("sgd3r2w")
    # ... and against the same probe run live on this GPU (stream_mix as a child process)
    live = r["plain_stream_ceiling_live"]
    assert "error" not in live, live
    assert live["case"].startswith("sgd3r2w") and 0.3 < live["frac"] < 1.0
    assert abs(r["frac_of_live_ceiling"] - r["frac"] / live["frac"]) < 1e-9
    # every beyond-cache row with an exact plain-stream mix carries its own live ceiling, the
    # 16-bit pack / unpack rows included
    lv = b["plain_stream_ceiling_live"]
    for row, mix in (("pack_bf16", "cvt16_16"), ("pack_f32_to_bf16", "cvt32_16"), ("unpack_bf16_to_f32", "cvt16_32"),
                     ("pack_f32", "copy"), ("sqnorm_f32", "read")):
        assert 0.3 < lv[mix]["frac"] < 1.0, (mix, lv.get(mix))
        assert abs(b["kernels"][row]["frac_of_live_ceiling"] - b["kernels"][row]["frac"] / lv[mix]["frac"]) < 1e-9
    if n == 1:  # configs[3]'s N>1 clip path at its N=8 shard, over the one-rank RCCL communicator
        z, zs = k["clip_path_zero_n8"], k["clip_path_zero_n8_scalar"]
        assert z["alg_bytes"] == 30 * z["shard_elems"] and z["avg_ms"] > 0 and z["kernels_ms"] > 0
        assert zs["avg_ms"] > 0 and z["vs_scalar_form"] > 0
    # the self-check step after the timed region (distributed_training_amd/parity.py)
    p = d["parity"]
    assert p is not None and p["ok"] is True and p["world"] == n, p
    assert p["averaged_grads"]["ok"] is True and p["weights_identical"] is True
    if n <= 2:  # bitwise at ws <= 2, the 4(n-1)*2^-24*sum|g|/n bound above
        assert p["averaged_grads"]["bitwise_equal"] is True
    assert p["buffers_identical"] is True


def test_bench_n1_contract(cuda_device):
    p = _run([sys.executable, "-u", "bench.py", "--gpus", "1"] + SMALL, _env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]
    _check_line(lines[0], 1)
    assert lines[0]["config"]["impl"] == "libgsync"
    assert lines[0]["parity"]["collective"] == "rccl(libgsync)"
    t = lines[0]["grad_sync"]["tail_ms"]  # last bucket ready -> every bucket chain done
    assert t["total"] > 0 and t["pack"] > 0 and t["collective"] >= 0 and t["unpack"] > 0
    assert t["total_timed_step"] > 0  # the timed steps' own tail (timeline level 1)
    assert len(lines[0]["grad_sync"]["bucket_timeline_ms"]) == lines[0]["grad_sync"]["n_buckets"]
    # BASELINE configs[3] and configs[4] in the N=1 line
    z = lines[0]["zero2"]
    assert z["engine"] == "zero2" and z["images_per_sec"] > 0 and z["parity"]["ok"] is True, z["parity"]
    assert 0 < z["shard_update"]["frac"] < 1.5
    c = lines[0]["colossal"]
    assert c["engine"] == "colossal" and c["images_per_sec"] > 0 and c["parity"]["ok"] is True, c["parity"]
    fa = c["fused_adam"]
    assert fa["launches"] + fa["skipped_launches"] == c["steps"]
    assert fa["launches"] == 0 or 0 < fa["frac"] < 1.5
    # configs[4] on torch alone in the same run (torch DDP + GradScaler + fused AdamW)
    assert c["torch"]["images_per_sec"] > 0 and c["torch"]["steps"] > 0
    assert abs(c["vs_torch"] - c["images_per_sec"] / c["torch"]["images_per_sec"]) < 1e-9


def test_bench_n2_driver_launch_gloo_rehearsal(cuda_device):
    env = _env()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "bench.py", "--gpus", "2", "--pg-backend", "gloo"] + SMALL
    p = _run(cmd, env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    _check_line(lines[0], 2)
    assert "rehearsal" in lines[0]["config"]
    assert lines[0]["parity"]["collective"] == "gloo"
    _check_policy_ab(lines[0], 2)
    # BASELINE configs[3] timed in the same N>1 run: the ZeRO-2 leg
    z = lines[0]["zero2"]
    assert z["engine"] == "zero2" and z["images_per_sec"] > 0 and z["shard_update"]["avg_launch_ms"] > 0
    assert z["parity"]["ok"] is True and z["parity"]["world"] == 2, z["parity"]
    c = lines[0]["colossal"]  # BASELINE configs[4] in the same run
    assert c["engine"] == "colossal" and c["images_per_sec"] > 0 and c["parity"]["ok"] is True, c["parity"]
    # the torch legs at N > 1 too: torch DDP over the same process group beside the headline
    t = lines[0]["torch_ddp"]
    assert t["images_per_sec"] > 0 and t["steps"] == 20
    assert abs(lines[0]["vs_baseline"] - lines[0]["value"] / t["images_per_sec"]) < 1e-9
    assert c["torch"]["images_per_sec"] > 0
    assert "leg_errors" not in lines[0], lines[0].get("leg_errors")


def _check_policy_ab(d, n):
    """The bucket-policy A/B the driver's N>1 run carries (DESIGN §8's rule
    decides row N1 from it): every variant timed, parity-checked, with its tail."""
    ab = d["bucket_policy_ab"]
    assert set(ab["variants"]) == {"torch", "xgmi", "last_bucket_cap_1MiB", "bf16_buckets", "rccl_cta_cap_16",
                                   "grad_as_bucket_view", "optimizer_overlap", "torch_again"}
    assert ab["decision"] != "bf16_buckets"
    for name, r in ab["variants"].items():
        assert r["images_per_sec"] > 0 and r["ms_per_step"] > 0, name
        assert r["parity"]["ok"] is True and r["parity"]["world"] == n, (name, r["parity"])
        assert r["tail_split_ms"] is None or r["tail_split_ms"]["total"] > 0
    assert ab["decision"] in ab["variants"]
    assert "rule" in ab and ab["torch_mean_images_per_sec"] > 0
    # the tail split caps the last bucket at 1 MiB: one more bucket than the torch layout
    assert len(ab["variants"]["last_bucket_cap_1MiB"]["bucket_bytes"]) >= len(ab["variants"]["torch"]["bucket_bytes"])
    if n > 1:
        assert ab["variants"]["xgmi"]["xgmi_calibration"]["bus_GBps"] > 0


def test_bench_policy_ab_n1_rccl(cuda_device):
    """The same A/B forced on at N=1 over libgsync's RCCL communicator (the
    comm-side code of the driver's run: re-wrapping, close(), the standalone leg)."""
    p = _run([sys.executable, "-u", "bench.py", "--gpus", "1", "--policy-ab", "1", "--kernel-rates", "0"] + SMALL + NO_LEGS,
             _env())
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_lines(p.stdout)[0]
    _check_policy_ab(d, 1)
    assert d["bucket_policy_ab"]["variants"]["torch"]["parity"]["collective"] == "rccl(libgsync)"


def test_bench_colossal_engine(cuda_device):
    """BASELINE configs[4]'s path: the Colossal Booster shim as run.sh drives it
    (TorchDDPPlugin, fp16 mixed precision, HybridAdam) through bench.py."""
    p = _run([sys.executable, "-u", "bench.py", "--gpus", "1", "--engine", "colossal", "--kernel-rates", "0"] + SMALL,
             _env())
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_lines(p.stdout)[0]
    assert d["config"]["engine"] == "colossal" and d["dtype"] == "fp16"
    assert d["roofline"]["algorithmic_bytes_per_launch"] == 28 * d["config"]["params"]
    # launches whose GradScaler step overflowed (the kernel exits on the device flag) are not counted
    assert d["roofline"]["launches"] + d["roofline"].get("skipped_launches", 0) == 3
    assert d["roofline"]["launches"] == 0 or d["roofline"]["achieved"] > 0
    assert d["parity"]["ok"] is True and d["parity"]["averaged_grads"]["bitwise_equal"] is True


@pytest.mark.parametrize("engine", ["ddp", "zero2"])
def test_bench_collective_bench_leg(cuda_device, engine):
    """The standalone collective leg the driver's N>1 runs take by default
    (`--collective-bench -1` = on when N>1), forced on at N=1 over libgsync's
    RCCL communicator: every bucket's all-reduce (DDP) or reduce-scatter +
    all-gather (ZeRO-2), the whole-gradient message and the 1-64 MiB curve;
    DDP with the overlapped optimizer, the parity step after it."""
    extra = ["--collective-bench", "1", "--kernel-rates", "0"] + NO_LEGS
    extra += ["--optimizer-overlap", "1"] if engine == "ddp" else ["--engine", "zero2"]
    p = _run([sys.executable, "-u", "bench.py", "--gpus", "1"] + SMALL + extra, _env())
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_lines(p.stdout)[0]
    sb = d["grad_sync"]["standalone"]
    ops = {r["op"] for r in sb["per_op"]}
    if engine == "ddp":
        assert {"all_reduce", "all_reduce_whole_grad", "all_reduce_1MiB", "all_reduce_64MiB"} <= ops
        assert d["config"]["optimizer_overlap"] is True
        assert d["grad_sync"]["tail_ms"]["total_timed_step"] > 0
    else:
        assert {"reduce_scatter", "all_gather"} <= ops
    assert all(r["median_ms"] > 0 for r in sb["per_op"])
    assert sb["xgmi_peak_GBps"] == 0 and sb["frac"] is None  # one rank: no link in use
    assert d["parity"]["ok"] is True and d["parity"]["collective"] == "rccl(libgsync)", d["parity"]


@pytest.mark.parametrize("engine,n", [("ddp", 4), ("zero2", 3)])
def test_bench_multirank_gloo_rehearsal(cuda_device, engine, n):
    """More ranks than the N=2 rehearsal, as the driver's 4/8-GPU runs: DDP at 4
    ranks (the parity step's ws > 2 tolerance path, rank order != the
    collective's order) and ZeRO-2 at 3 ranks (shards of a flat buffer padded
    to 3 x 64 elements; reduce-scatter / all-gather over the rehearsal group).  No torch
    legs: torch's own DDP over gloo stages every bucket through the host and alone
    takes most of the child's time limit at 4 ranks (the N=2 rehearsal runs them)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "bench.py", "--gpus", str(n), "--pg-backend", "gloo", "--kernel-rates", "0", "--torch-leg", "0"] + SMALL + NO_LEGS
    if engine == "zero2":
        cmd += ["--engine", "zero2"]
    # a healthy run takes ~30 s; a hung one dumps every rank's stacks each 40 s into the stderr file
    # (each dump also reaches the real stderr as a heartbeat) and fails at CHILD_LIMIT_S, inside the
    # box's 180 s silence window
    p = _run(cmd, dict(_env(), GSYNC_BENCH_TRACEBACK_S="40"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == 16 * n
    assert abs(d["value"] - n * 16 * 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    par = d["parity"]
    assert par["ok"] is True and par["world"] == n and par["collective"] == "gloo", par
    assert par["averaged_grads"]["ok"] is True and par["weights_identical"] is True
    if engine == "zero2":
        assert d["roofline"]["algorithmic_bytes_per_launch"] == 20 * (d["config"]["params"] // n)
    else:
        assert par["buffers_identical"] is True


def test_bench_wall_budget_skips_legs_keeps_the_headline(cuda_device):
    """N>1 with a wall budget already spent by warm-up (1 s): every optional leg
    is skipped and named in leg_errors, the headline and roofline intact, exit 0."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "bench.py", "--gpus", "2", "--pg-backend", "gloo", "--wall-budget-s", "1", "--kernel-rates", "0",
           "--policy-ab", "1"] + SMALL
    p = _run(cmd, _env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0 and d["n_gpus"] == 2
    skipped = {k for k, v in d["leg_errors"].items() if v.startswith("skipped")}
    assert {"tail_split", "parity", "collective_bench", "zero2", "colossal", "bucket_policy_ab",
            "torch_ddp"} <= skipped, skipped
    assert "legs_incomplete" not in d


def test_bench_leg_watchdog_exits_nonzero_keeps_the_headline(cuda_device):
    """N>1: a leg still running past the wall budget (a hung collective; here the
    test hook GSYNC_BENCH_TEST_HANG_LEG) ends every rank with exit status 3 after
    rank 0 printed the line — the headline and roofline intact, the leg named."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "bench.py", "--gpus", "2", "--pg-backend", "gloo", "--wall-budget-s", "1", "--kernel-rates", "0"] + SMALL
    env = dict(_env(), GSYNC_BENCH_TEST_HANG_LEG="parity")
    p = _run(cmd, env)
    assert p.returncode != 0, "a leg overrunning the budget must not look like a clean run"
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    assert d["legs_incomplete"] == {"leg": "parity", "wall_budget_s": 1.0}
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0 and d["n_gpus"] == 2
