#!/usr/bin/env python3
"""Plain `convert` shape on the device (generic kernels): one stream of B interleaved int16 bands covering the whole
raster (converter.py:185-216), device-resident; prints ms per encode and the profile buckets."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from flac_raster_amd import _native  # noqa: E402

B, H, W = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (4, 4096, 4096)))
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
ctx = _native.Context(0)
buf = ctx.alloc(B * H * W * 2)
ctx.synth_raster(buf, B, H, W, seed=5)
d = ctx.make_desc(H, W, np.int16, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16)
arena = ctx.alloc(ctx.arena_bound(d))
ctx.encode_tiles_device(buf.ptr, d, arena)
ctx.profile(True)
ctx.profile_reset()
ctx.sync()
t0 = time.perf_counter()
for _ in range(steps):
    off, mn, mx, bps = ctx.encode_tiles_device(buf.ptr, d, arena)
ctx.sync()
dt = (time.perf_counter() - t0) / steps
ctx.profile(False)
kern = {k: round(ctx.profile_avg_ms(k), 3) for k in ("stats", "analyze", "partial", "encode", "compact")}
print({"bands": B, "H": H, "W": W, "ms": round(dt * 1e3, 2), "Mpx_s": round(H * W / dt / 1e6, 1),
       "bytes": int(off[-1]), "kernels_ms": {k: v for k, v in kern.items() if v > 0}})
ctx.close()
