"""Multi-rank create-streaming: tile-row sharding + the size all-gather + pwritev assembly.

CPU tests run world-size 2 and 3 with the host exchange (TcpComm) and the oracle injected as the encoder; the GPU
variants run two ranks on the one GPU of the box with the HIP encoder (RCCL needs one GPU per rank, so they also
use the host exchange) and RCCL itself at world size 1.  Every variant must write the single-process file.
"""
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
TRANSFORM = [10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _band(H=700, W=650, seed=11):
    rng = np.random.default_rng(seed)
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    return (1000 + 300 * np.sin(x * 0.5) * np.cos(y * 0.3) + 50 * rng.random((H, W))).astype(np.int16)


def _oracle_encode(slab, tile):
    from flac_raster_amd.streaming import EncodedTiles, tile_grid
    from oracle import oracle as O
    arena, off, mn, mx = O.encode_tiles(slab, tile)
    return EncodedTiles(tile_grid(*slab.shape, tile), arena, off, mn, mx, 16)


def _worker(rank, world, port, out, band, tile, use_gpu):
    sys.path.insert(0, str(ROOT))
    from flac_raster_amd import distributed as D, geotiff
    comm = D.TcpComm(rank, world, "127.0.0.1", port)
    H, W = band.shape
    tr0, tr1 = D.shard_tile_rows((H + tile - 1) // tile, world, rank)
    slab = np.ascontiguousarray(band[tr0 * tile:min(tr1 * tile, H)])
    ctx = None
    if use_gpu:
        from flac_raster_amd import _native
        ctx = _native.Context(0)
        encode = D.gpu_encoder(ctx)
    else:
        encode = _oracle_encode
    D.create_streaming_sharded(slab, tr0 * tile, (H, W), geotiff.Affine(*TRANSFORM), "EPSG:32636", tile, Path(out),
                               comm, encode)
    comm.close()
    if ctx is not None:
        ctx.close()


def _run_ranks(world, out, band, tile, use_gpu=False):
    port = _free_port()
    ctxm = mp.get_context("spawn")
    procs = [ctxm.Process(target=_worker, args=(r, world, port, str(out), band, tile, use_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _reference(band, tile):
    from oracle import pipeline as P
    return P.create_streaming(band, TRANSFORM + [0.0, 0.0, 1.0], "EPSG:32636", tile)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_create_streaming_matches_single_process(tmp_path, world):
    band = _band()
    out = tmp_path / "sharded.flac"
    out.write_bytes(b"x" * 5_000_000)  # a larger stale file: the ranks never truncate below their data
    _run_ranks(world, out, band, 256)
    assert out.read_bytes() == _reference(band, 256)


def test_shard_tile_rows_balanced():
    from flac_raster_amd.distributed import shard_tile_rows
    parts = [shard_tile_rows(79, 8, r) for r in range(8)]
    assert parts[0][0] == 0 and parts[-1][1] == 79
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    assert {p[1] - p[0] for p in parts} <= {9, 10}


def test_tcp_allgather_variable_sizes():
    from flac_raster_amd.distributed import all_gather_sizes

    class Fake:  # world 1
        rank, world = 0, 1

        @staticmethod
        def allgather_i64(a):
            return np.asarray(a)

    assert list(all_gather_sizes(np.array([5, 6]), [2], Fake())) == [5, 6]


@pytest.mark.gpu
def test_sharded_two_ranks_gpu_encoder(tmp_path):
    band = _band(1100, 900, 5)
    out = tmp_path / "sharded_gpu.flac"
    _run_ranks(2, out, band, 256, use_gpu=True)
    assert out.read_bytes() == _reference(band, 256)


@pytest.mark.gpu
def test_rccl_comm_world_one(gpu_ctx, tmp_path, monkeypatch):
    """RCCL through the C-ABI (frs_comm_*): a world-1 communicator all-gathers and drives the sharded writer."""
    from flac_raster_amd import distributed as D, geotiff
    monkeypatch.setenv("FRS_COMM_PORT", str(_free_port()))
    comm = D.init_comm(gpu_ctx, "rccl", rank=0, world=1)
    try:
        assert list(comm.allgather_i64(np.array([3, -1, 2 ** 40]))) == [3, -1, 2 ** 40]
        band = _band()
        out = tmp_path / "rccl1.flac"
        D.create_streaming_sharded(band, 0, band.shape, geotiff.Affine(*TRANSFORM), "EPSG:32636", 256, out, comm,
                                   D.gpu_encoder(gpu_ctx))
    finally:
        comm.close()
    assert out.read_bytes() == _reference(band, 256)


def test_more_ranks_than_tile_rows(tmp_path):
    """World 3 on a band of one tile row: ranks 1 and 2 hold empty slabs, still join the exchange, and the file is
    the single-process one."""
    band = _band(200, 650, 3)
    out = tmp_path / "tiny.flac"
    _run_ranks(3, out, band, 256)
    assert out.read_bytes() == _reference(band, 256)


_HANG_SCRIPT = """
import os, sys, time
sys.path.insert(0, {root!r})
from flac_raster_amd import distributed as D
rank, world, _ = D.env_rank_world()
if rank == 1:
    sys.exit(3)             # a rank that dies before the exchange
comm = D.init_comm(None, "tcp")
comm.barrier()              # rank 0 would wait here for the dead peer
time.sleep(600)
"""


def test_rank_failure_is_bounded(tmp_path):
    """launch.run_ranks: one rank exits non-zero -> the group stops within seconds and returns that code."""
    import time
    from flac_raster_amd import launch
    script = tmp_path / "hang.py"
    script.write_text(_HANG_SCRIPT.format(root=str(ROOT)))
    t0 = time.monotonic()
    rc = launch.run_ranks(2, [str(script)], module=None, timeout=60)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_cli_create_streaming_gpus_failure_returns_1(tmp_path):
    """create-streaming --gpus 2 whose ranks cannot run (no GPU here; one GPU on the test box) exits 1 promptly."""
    import subprocess
    import time
    from flac_raster_amd import geotiff
    src = tmp_path / "in.tif"
    geotiff.write(src, _band(300, 300, 2), geotiff.Affine(*TRANSFORM), 32636)
    t0 = time.monotonic()
    env = dict(os.environ, FRS_COMM_TIMEOUT="20")
    r = subprocess.run([sys.executable, "-m", "flac_raster_amd", "create-streaming", str(src), "-o",
                        str(tmp_path / "o.flac"), "--tile-size", "128", "--gpus", "2"], cwd=str(ROOT), env=env,
                       capture_output=True, timeout=120)
    assert r.returncode == 1, r.stderr[-2000:]
    assert time.monotonic() - t0 < 30


def test_bench_gpus_n_launches_n_ranks():
    """bench.py --gpus 2 without a launcher starts two ranks (the driver's command shape); the self-test mode
    exchanges rank ids over the host all-gather and rank 0 reports n_gpus 2."""
    import json
    import subprocess
    env = dict(os.environ, FRS_BENCH_SELFTEST="1", FRS_COMM_BACKEND="tcp")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       timeout=120, text=True)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1]
    assert "host TCP" in line["config"]["parallelism"]
    bad = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=dict(env, WORLD_SIZE="1"),
                         capture_output=True, timeout=60, text=True)
    assert bad.returncode != 0
