"""Local multi-GPU launcher: one process per GPU, each a rank of the sharded create-streaming.

``flac-raster create-streaming in.tif -o out.flac --gpus 8`` re-runs the command in N child processes with the
launcher environment a torchrun-style tool would set (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT);
each child drives its own GPU (LOCAL_RANK) and the ranks exchange tile sizes over RCCL (distributed.py).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(n: int, argv: List[str]) -> int:
    """Start `n` ranks of ``python -m flac_raster_amd <argv>``; returns the first non-zero exit code (or 0)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FRS_COMM_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-m", "flac_raster_amd"] + argv, env=env))
    rc = 0
    for p in procs:
        code = p.wait()
        rc = rc or code
    return rc
