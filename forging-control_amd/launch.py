"""One process per GPU for a single-node data-parallel run, started BEFORE anything touches the GPU.

``python bench.py --gpus N`` (or any script following the same pattern) calls :func:`spawn_ranks` when no
``WORLD_SIZE`` is set: it starts ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 ...`` on the same script and arguments as a CHILD process and returns its exit
code. Each rank then finds RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in its environment, binds
``cuda:LOCAL_RANK`` and joins the RCCL (or gloo) process group. The parent never initialises HIP, so
no process that has touched the GPU is ever replaced by another program.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nprocs: int, script: str, argv: list[str], port: int | None = None,
                extra_env: dict | None = None, timeout: float | None = None) -> int:
    """Run ``script argv`` as ``nprocs`` ranks of one node (torchrun, rendezvous on 127.0.0.1) and return
    the launcher's exit code (non-zero if any rank failed)."""
    if nprocs < 1:
        raise ValueError(f"nprocs must be >= 1, got {nprocs}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr", "127.0.0.1", f"--master-port={port or free_port()}", script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC: RCCL peer buffers across processes
    env.setdefault("OMP_NUM_THREADS", "1")
    env.update(extra_env or {})
    return subprocess.run(cmd, env=env, timeout=timeout).returncode


def rank_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) of this process (1 rank when launched directly)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
