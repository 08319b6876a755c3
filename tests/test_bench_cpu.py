"""bench.py / bench_kernels.py / scripts compile and parse their arguments
without a GPU (the driver runs bench.py unattended on the box: a syntax or
argument error there costs a whole round's measurement)."""
import os
import py_compile
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", ["bench.py", "bench_kernels.py", "__graft_entry__.py", "scripts/kernel_only.py",
                                  "scripts/pmc_traffic.py", "scripts/overlap.py"])
def test_compiles(path):
    py_compile.compile(os.path.join(REPO, path), doraise=True)


def test_bench_defaults_parse():
    code = ("import sys; sys.argv=['bench.py']; sys.path.insert(0, %r); import bench; a = bench.parse(); "
            "assert a.gpus == 1 and a.steps == 20 and a.warmup == 5 and a.engine == 'ddp' and a.parity == 1; "
            "print('ok')" % REPO)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]


@pytest.mark.parametrize("script", sorted(f for f in os.listdir(os.path.join(REPO, "scripts")) if f.endswith(".sh")))
def test_gpu_scripts_parse(script):
    p = subprocess.run(["bash", "-n", os.path.join(REPO, "scripts", script)], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_every_script_is_cited():
    """Each script kept under scripts/ is cited by DESIGN.md, README.md or a test
    (one-offs that are not go to scripts/archive/, provenance of older profiles)."""
    import glob
    import re

    text = "".join(open(os.path.join(REPO, f)).read() for f in ("DESIGN.md", "README.md", "INTEGRATION.md", "bench.py"))
    text += "".join(open(f).read() for f in glob.glob(os.path.join(REPO, "tests", "*.py")))
    text += "".join(open(f).read() for f in glob.glob(os.path.join(REPO, "scripts", "*.sh")))
    for f in sorted(os.listdir(os.path.join(REPO, "scripts"))):
        path = os.path.join(REPO, "scripts", f)
        if os.path.isdir(path) or f.startswith("."):
            continue
        assert re.search(r"(?<![A-Za-z0-9_])" + re.escape(f), text), f"scripts/{f} is cited nowhere"


def test_leg_cost_scales_with_world_size():
    """The wall-budget skip rule's leg estimates grow with the ranks:
    at one GPU per rank by the per-rank growth and communicator set-up, under the gloo
    rehearsal by the ranks sharing each GPU as well."""
    code = ("import sys; sys.argv=['bench.py']; sys.path.insert(0, %r); import bench\n"
            "for leg in bench.LEG_COST_S:\n"
            "    c1 = bench.leg_cost(leg, 1, 'nccl')\n"
            "    c8 = bench.leg_cost(leg, 8, 'nccl')\n"
            "    g8 = bench.leg_cost(leg, 8, 'gloo', ranks_per_gpu=8)\n"
            "    f7 = 7 * bench.LEG_FIXED_PER_RANK_S.get(leg, 0.0)\n"
            "    assert abs(bench.leg_cost(leg, 8, 'gloo', 8, batch=64) - max(5.0, (g8 - f7) / 4 + f7)) < 1e-9 "
            "or g8 == 5.0, leg\n"
            "    assert c1 == max(5.0, bench.LEG_COST_S[leg]), leg\n"
            "    assert c8 >= c1 * (1 + 7 * bench.LEG_GROWTH_PER_RANK) - 1e-9 or c8 == 5.0, leg\n"
            "    assert g8 >= 8 * c8 - 8 * 7 * bench.LEG_FIXED_PER_RANK_S.get(leg, 0.0) - 1e-9 or g8 == 5.0, leg\n"
            "# torch's own DDP legs stage through the host under gloo (the 8-rank rehearsal, r6n8c)\n"
            "for leg, f in bench.LEG_GLOO_FACTOR.items():\n"
            "    assert f >= 1 and leg in bench.LEG_COST_S, leg\n"
            "    assert abs(bench.leg_cost(leg, 8, 'gloo', 8, batch=64) - f * bench.LEG_COST_S[leg] * 2 * 1.7) < 1e-9, leg\n"
            "    assert abs(bench.leg_cost(leg, 8, 'nccl') - bench.LEG_COST_S[leg] * 1.7) < 1e-9, leg\n"
            "print('ok')" % REPO)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]


def test_every_profile_is_cited():
    """Each record kept under profiles/ is cited (by path, file name or its directory) by
    DESIGN.md, README.md, INTEGRATION.md, bench.py, a test, a script, a native source or
    a directory's INDEX.md; superseded records leave the tree for profiles/ARCHIVE.md's index (VERDICT
    r5 next 9)."""
    import glob
    import re

    srcs = ["DESIGN.md", "README.md", "INTEGRATION.md", "bench.py", "bench_kernels.py", "__graft_entry__.py"]
    srcs += glob.glob(os.path.join(REPO, "tests", "*.py")) + glob.glob(os.path.join(REPO, "scripts", "*.sh"))
    srcs += glob.glob(os.path.join(REPO, "scripts", "*.py")) + glob.glob(os.path.join(REPO, "profiles", "**", "INDEX.md"),
                                                                         recursive=True)
    srcs += [f for f in glob.glob(os.path.join(REPO, "distributed_training_amd", "csrc", "*")) if os.path.isfile(f)]
    text = "".join(open(s if os.path.isabs(s) else os.path.join(REPO, s), errors="replace").read() for s in srcs)
    missing = []
    for root, _, names in os.walk(os.path.join(REPO, "profiles")):
        for n in names:
            rel = os.path.relpath(os.path.join(root, n), REPO)
            if n in ("ARCHIVE.md", "INDEX.md") or n.startswith("."):
                continue
            if rel in text or rel[len("profiles/"):] in text or re.search(r"(?<![\w/])" + re.escape(n), text):
                continue
            d, ok = os.path.dirname(rel), False
            while d not in ("profiles", ""):
                if re.search(re.escape(d) + r"(/|\b)", text):
                    ok = True
                    break
                d = os.path.dirname(d)
            if not ok:
                missing.append(rel)
    assert not missing, f"{len(missing)} uncited profile records, e.g. {missing[:10]}"
