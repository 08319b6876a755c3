"""The drop-in boundary is a C ABI: a plain C program (tests/c_abi/host_roundtrip.c)
compiled with gcc against include/gsync.h and linked to libgsync.so drives
host plans (pack / unpack / Σg² / SGD), the sampler and the error path,
without Python or torch in the process."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "distributed_training_amd", "lib")


def test_plain_c_caller(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libgsync.so")):
        pytest.skip("libgsync.so not built")
    exe = tmp_path / "host_roundtrip"
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c_abi", "host_roundtrip.c"), "-o", str(exe),
                    "-L", LIBDIR, "-lgsync", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib",
                    "-Wl,--allow-shlib-undefined", "-lm"], check=True)
    env = dict(os.environ, LD_LIBRARY_PATH=f"/opt/rocm/lib:{os.environ.get('LD_LIBRARY_PATH', '')}")
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=60)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
