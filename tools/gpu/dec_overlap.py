"""Round 6 experiment: can two halves of the batched C4 decode overlap on two streams (two contexts, two host
threads)?  The lane decoder is VALU-latency-bound, the span check LDS-bound and the selection HBM-bound, so a
half's decode might hide under the other half's selection and span check.
usage: python tools/gpu/dec_overlap.py [reps]   (one JSON line)"""
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from flac_raster_amd import _native, streaming  # noqa: E402


class View:  # a DeviceBuffer-like window (ptr, nbytes) into another buffer
    def __init__(self, ptr, nbytes):
        self.ptr, self.nbytes = ptr, nbytes


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    H = W = 40000
    B, T = 4, 512
    ctx = _native.Context(0)
    ctx2 = _native.Context(0)
    raster = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(raster, B, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    counts = [w * h for (_, _, w, h) in streaming.tile_grid(H, W, T)]
    n = len(counts)
    out = ctx.alloc(H * W * 2)
    h = n // 2
    px_h = int(sum(counts[:h]))

    def full():
        ctx.decode_tiles_device(arena, off, counts, 1, 16, mn, mx, np.int16, out)

    def half(c, lo, hi, obase):
        c.decode_tiles_device(arena, off[lo:hi + 1] - off[lo], counts[lo:hi], 1, 16, mn[lo:hi], mx[lo:hi], np.int16,
                              View(out.ptr + obase, out.nbytes - obase), blob_ptr=arena.ptr + int(off[lo]))

    def halves_seq():
        half(ctx, 0, h, 0)
        half(ctx, h, n, px_h * 2)

    def halves_par():
        t = threading.Thread(target=half, args=(ctx2, h, n, px_h * 2))
        t.start()
        half(ctx, 0, h, 0)
        t.join()

    res = {}
    for name, fn in (("full", full), ("halves_seq", halves_seq), ("halves_par", halves_par)) * 2:
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        res.setdefault(name, []).append(round(min(ts), 3))
    # the halves' output equals the full decode's
    ref = out.download(H * W * 2).copy()
    halves_par()
    res["par_equal_full"] = bool(np.array_equal(out.download(H * W * 2), ref))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
