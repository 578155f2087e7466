"""World-size-2 gloo test of the tile-row sharding + size all-gather + pwrite assembly.

The encoder is injected: the CPU oracle stands in for the GPU codec here (tests only); the GPU path
uses the same function with the HIP encoder (bench.py, -m gpu tests).
"""
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_encode(slab, tile):
    from flac_raster_amd.streaming import EncodedTiles, tile_grid
    from oracle import oracle as O
    arena, off, mn, mx = O.encode_tiles(slab, tile)
    return EncodedTiles(tile_grid(*slab.shape, tile), arena, off, mn, mx, 16)


def _worker(rank, world, port, out, band, tile):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from flac_raster_amd import distributed as D, geotiff
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W = band.shape
    trows = (H + tile - 1) // tile
    tr0, tr1 = D.shard_tile_rows(trows, world, rank)
    slab = np.ascontiguousarray(band[tr0 * tile:min(tr1 * tile, H)])
    t = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    D.create_streaming_sharded(slab, tr0 * tile, (H, W), t, "EPSG:32636", tile, Path(out), dist, _oracle_encode)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_create_streaming_matches_single_process(tmp_path, world):
    rng = np.random.default_rng(11)
    H, W, tile = 700, 650, 256
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    band = (1000 + 300 * np.sin(x * 0.5) * np.cos(y * 0.3) + 50 * rng.random((H, W))).astype(np.int16)
    out = tmp_path / "sharded.flac"
    mp.spawn(_worker, args=(world, _free_port(), str(out), band, tile), nprocs=world, join=True)
    from oracle import pipeline as P
    ref = P.create_streaming(band, [10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0, 0.0, 0.0, 1.0], "EPSG:32636", tile)
    assert out.read_bytes() == ref


def test_shard_tile_rows_balanced():
    from flac_raster_amd.distributed import shard_tile_rows
    parts = [shard_tile_rows(79, 8, r) for r in range(8)]
    assert parts[0][0] == 0 and parts[-1][1] == 79
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    assert {p[1] - p[0] for p in parts} <= {9, 10}
