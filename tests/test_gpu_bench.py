"""bench.py's N > 1 line rehearsed on one GPU (the tile loop cli.py:690-763 sharded by tile rows).

The driver runs `bench.py --gpus N` on an 8-GPU node; this box has one GPU, so two ranks share it over the host
exchange (FRS_COMM_BACKEND=tcp).  The line must carry n_gpus, the all-gather figures reported apart from the
encode, and the same compressed bytes as the single-rank run of the same raster (the shards are the same tiles).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
ARGS = ["--height", "4096", "--width", "4096", "--no-extras", "--no-cpu", "--queries", "50", "--steps", "3",
        "--warmup", "1"]


def _bench(gpus: int) -> dict:
    env = dict(os.environ, FRS_COMM_BACKEND="tcp", FRS_COMM_TIMEOUT="60")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", str(gpus), *ARGS], env=env,
                       capture_output=True, text=True, timeout=240, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_bench_two_ranks_reports_allgather_and_same_bytes():
    one = _bench(1)
    two = _bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert "allgather_us" not in one
    ag = two["allgather_us"]
    for k in ("in_step", "isolated"):
        assert set(ag[k]) == {"mean", "max", "p50"} and ag[k]["mean"] > 0 and ag[k]["max"] >= ag[k]["p50"]
    assert ag["steps"] == 3
    assert two["config"]["compressed_bytes_total"] == one["config"]["compressed_bytes_total"] > 0
    assert two["config"]["tiles"] == one["config"]["tiles"] == 64
    assert two["bbox_extract"]["queries"] == one["bbox_extract"]["queries"] == 50
    assert two["bbox_extract"]["lossless"] and one["bbox_extract"]["lossless"]
