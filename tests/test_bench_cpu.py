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
