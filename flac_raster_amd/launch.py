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
import time
from typing import List, Optional


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(n: int, argv: List[str], timeout: Optional[float] = None, module: Optional[str] = "flac_raster_amd",
              extra_env: Optional[dict] = None) -> int:
    """Start `n` ranks of ``python -m <module> <argv>`` (module None: ``python <argv>``) and wait for all of them.

    The children are polled together: as soon as one exits non-zero the others are terminated (then killed after
    a grace period) and that exit code is returned -- a rank that fails after the communicator is up would
    otherwise leave its peers blocked in the all-gather.  `timeout` (seconds) bounds the whole run (exit 124)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FRS_COMM_PORT=str(port), **(extra_env or {}))
        cmd = [sys.executable] + (["-m", module] if module else []) + list(argv)
        procs.append(subprocess.Popen(cmd, env=env))
    t_end = None if timeout is None else time.monotonic() + timeout
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        if all(c == 0 for c in codes):
            return 0
        if t_end is not None and time.monotonic() > t_end:
            rc = 124
            break
        time.sleep(0.05)
    _stop(procs)
    return rc


def _stop(procs, grace: float = 5.0) -> None:
    for p in procs:
        if p.poll() is None:
            p.terminate()
    t_end = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, t_end - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
