"""The drop-in boundary on the GPU without Python in the loop: a plain C
program (tests/c_abi/hip_bucketer.c, gcc + the HIP runtime's C API, built by
__graft_entry__.build() / tests/c_abi/Makefile) creates an RCCL communicator,
computes torch's bucket assignment, drives the bucketer through
prepare / mark_ready per gradient on a HIP stream / finalize, and runs two
fused SGD steps — checked in the same process against the C oracle
(averaged grads and the SGD state bit for bit, Σg² to 1e-5)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "c_abi", "build", "hip_bucketer")


@pytest.mark.gpu
def test_plain_c_bucketer_on_gpu(cuda_device):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "c_abi")], check=True, timeout=120)
    env = dict(os.environ, LD_LIBRARY_PATH=f"/opt/rocm/lib:{os.environ.get('LD_LIBRARY_PATH', '')}")
    out = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=120)
    last = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else ""  # after RCCL's banner
    assert out.returncode == 0 and last.startswith("ok"), out.stdout[-2000:] + out.stderr[-2000:]
