#!/usr/bin/env python3
"""The bench's Sentinel-2 workload alone (10980^2 uint16, tile 1024, device-resident), for kernel traces."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from flac_raster_amd import _native  # noqa: E402

ctx = _native.Context(0)
print(bench.sentinel2(ctx, steps=int(sys.argv[1]) if len(sys.argv) > 1 else 3))
ctx.close()
