"""Helpers for multi-process tests (gloo on CPU, or on one GPU)."""
import os
import random
import socket


def free_port():
    for _ in range(50):
        p = random.randint(20000, 45000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
                return p
            except OSError:
                continue
    raise RuntimeError("no free port")


def init_pg(backend, rank, ws, port):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=ws)
