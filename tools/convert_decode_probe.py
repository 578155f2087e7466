#!/usr/bin/env python3
"""flac_to_tiff shape on the device: encode a B-band raster as one stream (plain convert), then decode + de-normalise
the whole stream in one frs_decode_tiles_device call; prints ms and the decode buckets, checks the round trip."""
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
off, mn, mx, _ = ctx.encode_tiles_device(buf.ptr, d, arena)
out = ctx.alloc(B * H * W * 2)
args = (arena, np.array([0, off[-1]]), [H * W], B, 16, [mn[0]], [mx[0]], np.int16, out)
ctx.decode_tiles_device(*args)
ctx.profile(True)
ctx.profile_reset()
ctx.sync()
t0 = time.perf_counter()
for _ in range(steps):
    ctx.decode_tiles_device(*args)
ctx.sync()
dt = (time.perf_counter() - t0) / steps
ctx.profile(False)
kern = {k: round(ctx.profile_avg_ms(k), 3) for k in ("decode", "decode_span", "decode_frames", "decode_wave")}
# round trip: the decoded interleaved samples vs the raster (lossless)
got = out.download(B * H * W * 2).view(np.int16).reshape(H * W, B)
ref = buf.download(B * H * W * 2).view(np.int16).reshape(B, H * W).T
print({"bands": B, "H": H, "W": W, "ms": round(dt * 1e3, 2), "Mpx_s": round(H * W / dt / 1e6, 1),
       "kernels_ms": {k: v for k, v in kern.items() if v > 0}, "lossless": bool(np.array_equal(got, ref))})
ctx.close()
