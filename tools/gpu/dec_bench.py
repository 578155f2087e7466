"""Decode-only timing on the C4 arena: batched decode of all tiles (reps) and C5 bbox queries, as in bench.py.

usage: python tools/gpu/dec_bench.py [reps] [queries]   (prints one JSON line)
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from flac_raster_amd import _native  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    H = W = 40000
    B, T = 4, 512
    ctx = _native.Context(0)
    raster = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(raster, B, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    res = {}
    bd = [bench.batched_decode(ctx, arena, off, mn, mx, H, W, T) for _ in range(reps)]
    res["batched_decode"] = bd
    if nq:
        res["bbox_extract"] = bench.bbox_extract(ctx, None, raster, arena, off, mn, mx, H, W, T, 0, [len(off) - 1], nq)
    print(json.dumps(res), flush=True)
    arena.close()
    raster.close()
    ctx.close()


if __name__ == "__main__":
    main()
