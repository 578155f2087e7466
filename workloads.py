"""Benchmark/test workloads of BASELINE.json shared by bench.py and tests/ -- not product code.

C3/C4: [4][H][W] int16 synthetic DEM rasters generated on the device (frs_synth_raster_device), band 1 encoded
at tile 512.  C5: bbox queries against the C4 streaming index, rng seed 7, uniform tile centre, side
U[0.1, 2.0] * tile_size * pixel, clipped to the raster (from_origin(500000, 4000000, 10, 10), EPSG:32636).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

PIXEL = 10.0
LEFT, TOP = 500000.0, 4000000.0
CRS = "EPSG:32636"


def transform():
    from flac_raster_amd import geotiff
    return geotiff.Affine(PIXEL, 0.0, LEFT, 0.0, -PIXEL, TOP)


def streaming_index(rows: int, width: int, tile: int, tile_bytes: Sequence[int], row0: int = 0) -> Dict:
    """The create-streaming index (cli.py:679-686, 748-759) of a rows x width raster whose tile i holds
    tile_bytes[i] bytes; byte offsets are cumulative."""
    from flac_raster_amd import streaming
    tr = transform()
    frames: List[Dict] = []
    off = 0
    for i, (col, row, w, h) in enumerate(streaming.tile_grid(rows, width, tile)):
        _, bb = streaming.tile_transform_and_bbox(tr, col, row + row0, w, h)
        n = int(tile_bytes[i])
        frames.append({"frame_id": i, "bbox": bb, "window": {"col_off": col, "row_off": row + row0, "width": w,
                                                            "height": h}, "byte_offset": off, "byte_size": n})
        off += n
    return {"crs": CRS, "transform": list(tr) + [0.0, 0.0, 1.0], "width": width, "height": rows, "tile_size": tile,
            "frames": frames}


def c5_queries(rows: int, width: int, tile: int, n: int, seed: int = 7) -> List[List[float]]:
    """n bbox queries: tile-aligned uniform centre, side U[0.1, 2.0] tile sizes, clipped."""
    from flac_raster_amd import streaming
    grid = streaming.tile_grid(rows, width, tile)
    right, bottom = LEFT + width * PIXEL, TOP - rows * PIXEL
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        col, row, w, h = grid[int(rng.integers(len(grid)))]
        cx, cy = LEFT + (col + w / 2) * PIXEL, TOP - (row + h / 2) * PIXEL
        half = rng.uniform(0.1, 2.0) * tile * PIXEL / 2
        out.append([max(LEFT, cx - half), max(bottom, cy - half), min(right, cx + half), min(TOP, cy + half)])
    return out


def oracle_threads() -> int:
    """CPU threads for oracle legs: the box's CPU share (OMP_NUM_THREADS is set to it on the GPU box)."""
    import os
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
