#!/usr/bin/env python3
"""Batched-decode probe (profiling aid): encode a synthetic H x W int16 band at tile 512 on the device, then decode
every tile in one fused call `reps` times.  Under rocprofv3 the decode kernels dominate the trace."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from flac_raster_amd import _native, streaming
    H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    T = 512
    ctx = _native.Context(0)
    ras = ctx.alloc(H * W * 2)
    ctx.synth_raster(ras, 1, H, W, seed=1234)
    d = ctx.make_desc(H, W, np.int16, tile_h=T, tile_w=T)
    arena = ctx.alloc(ctx.arena_bound(d))
    off, mn, mx, _ = ctx.encode_tiles_device(ras.ptr, d, arena)
    counts = [w * h for (_, _, w, h) in streaming.tile_grid(H, W, T)]
    out = ctx.alloc(H * W * 2)
    ctx.profile(True)
    for r in range(reps):
        ctx.sync()
        t0 = time.perf_counter()
        ctx.decode_tiles_device(arena, off, counts, channels=1, bps=16, data_min=mn, data_max=mx, dtype=np.int16,
                                out=out)
        ctx.sync()
        print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    print({k: round(ctx.profile_avg_ms(k), 3) for k in ("decode", "decode_span", "decode_frames",
                                                          "lane_fallback_frames")})
    back = np.empty(H * W, np.int16)
    out.download(H * W * 2, 0, out=back.view(np.uint8))
    band = np.empty(H * W, np.int16)
    ras.download(H * W * 2, 0, out=band.view(np.uint8))
    print("first tile lossless:", bool(np.array_equal(back[:T * T].reshape(T, T), band.reshape(H, W)[:T, :T])))


if __name__ == "__main__":
    main()
