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


@pytest.mark.parametrize("script", ["gpu_round.sh", "gpu_tests.sh", "r2_tail.sh", "red_sweep.sh"])
def test_gpu_scripts_parse(script):
    p = subprocess.run(["bash", "-n", os.path.join(REPO, "scripts", script)], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
