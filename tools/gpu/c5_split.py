"""Round 6 experiment: where the C5 pipe decode's ~103 us go -- the same 300 queries decoded into page-locked host
memory (the bench's form) and into device memory, kernel times from the library's profile events.
usage: python tools/gpu/c5_split.py   (one JSON line)"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import workloads  # noqa: E402
from flac_raster_amd import _native, streaming  # noqa: E402


def main():
    H = W = 40000
    B, T = 4, 512
    ctx = _native.Context(0)
    raster = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(raster, B, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    index = workloads.streaming_index(H, W, T, np.diff(off))
    queries = workloads.c5_queries(H, W, T, 300)
    picks = []
    for q in queries:
        f = streaming.first_intersecting(index, q)
        picks.append((f["frame_id"], f["window"]["width"] * f["window"]["height"]))
    res = {}
    for name, out in (("host", ctx.host_buffer(T * T * 2)), ("device", ctx.alloc(T * T * 2))) * 2:
        for i, n in picks[:20]:
            ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, mn[i], mx[i], np.int16, out)
        lat = []
        for i, n in picks:
            t0 = time.perf_counter()
            ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, mn[i], mx[i], np.int16, out)
            lat.append(time.perf_counter() - t0)
        ctx.sync()
        ctx.profile(True)
        ctx.profile_reset()
        for i, n in picks[:100]:
            ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, mn[i], mx[i], np.int16, out)
        ctx.sync()
        ctx.profile(False)
        res.setdefault(name, []).append({"p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 4),
                                         "decode": round(ctx.profile_avg_ms("decode"), 4),
                                         "decode_frames": round(ctx.profile_avg_ms("decode_frames"), 4)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
