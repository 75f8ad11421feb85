"""Single-node launcher: one process per GPU over RCCL/xGMI.

``python -m multigrad_amd.launch -n 8 script.py [args...]`` starts ``-n`` ranks with
``torch.distributed.run`` (rendezvous on 127.0.0.1), sets ``LOCAL_RANK``/``RANK``/
``WORLD_SIZE`` for :func:`multigrad_amd.init_distributed`, and keeps
``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC) in the environment of every rank.  It
replaces ``mpiexec -n N python ...`` from the reference's docs; the launcher starts the
ranks as child processes and exits with their status.
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def build_command(nproc: int, script: str, args, port: int, nnodes: int = 1) -> list:
    return [sys.executable, "-m", "torch.distributed.run", f"--nnodes={nnodes}",
            f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            script] + list(args)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nproc", type=int, default=None,
                    help="ranks (default: number of visible GPUs, else 1)")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    n = a.nproc
    if n is None:
        import torch
        n = max(1, torch.cuda.device_count())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MULTIGRAD_PROGRESS", env.get("MULTIGRAD_PROGRESS", "1"))
    cmd = build_command(n, a.script, a.args, a.port or _free_port())
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
