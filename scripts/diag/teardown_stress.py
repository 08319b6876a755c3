"""Diagnostic: run a CPU/gloo world-size-2 DDP worker many times WITHOUT the
tests' os._exit shortcut and with a terminate/SIGABRT backtrace handler
(build/libterminate_trace.so from scripts/diag/terminate_trace.cpp), to name
the destructor behind the occasional exit-time abort.

    python scripts/diag/teardown_stress.py [runs] [fn]
"""
import ctypes
import os
import sys
import time

import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def worker(fn_name, rank, ws, port):
    ctypes.CDLL(os.path.join(REPO, "build", "libterminate_trace.so"))
    import faulthandler

    faulthandler.enable(all_threads=True)
    from tests import test_ddp_cpu as T
    from tests._dist_util import init_pg

    import torch
    import torch.distributed as dist

    init_pg("gloo", rank, ws, port)
    torch.set_num_threads(max(1, 8 // ws))
    getattr(T, fn_name)(rank, ws)
    if os.environ.get("NO_DESTROY", "0") == "0":  # as tests/test_ddp_cpu.py:_wrap
        dist.barrier()
        dist.destroy_process_group()
    # normal interpreter exit from here (atexit, module teardown, static destructors)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    fn = sys.argv[2] if len(sys.argv) > 2 else "_unused_across_ranks"
    from tests._dist_util import free_port

    ctx = mp.get_context("spawn")
    bad = 0
    t0 = time.time()
    for i in range(runs):
        port = free_port()
        ps = [ctx.Process(target=worker, args=(fn, r, 2, port)) for r in range(2)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
        codes = [p.exitcode for p in ps]
        if any(c != 0 for c in codes):
            bad += 1
            print(f"run {i}: exit codes {codes}", flush=True)
    print(f"{bad}/{runs} runs with a non-zero exit ({time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
