"""C5 query latency breakdown on the C4 arena: selection (host), decode call (device + sync), result download."""
import ctypes
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
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    H = W = 40000
    T = 512
    ctx = _native.Context(0)
    raster = ctx.alloc(4 * H * W * 2)
    ctx.synth_raster(raster, 4, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    index = workloads.streaming_index(H, W, T, np.diff(off))
    qs = workloads.c5_queries(H, W, T, nq)
    out = ctx.alloc(T * T * 2)
    host = ctx.pinned(T * T * 2).view(np.int16)
    ts, td, tc = [], [], []
    mode = sys.argv[2] if len(sys.argv) > 2 else ""
    prof = mode == "prof"  # kernel times (the profile's events add ~10 us per kernel)
    hostout = mode.startswith("hostout")
    one = mode == "hostout1"
    old1 = mode == "hostout1old"
    tabs = ((ctypes.c_int64 * 2)(), (ctypes.c_int64 * 2)(), (ctypes.c_double * 1)(), (ctypes.c_double * 1)())  # + the single-stream call (decode_tile_device: reused ctypes tables)  # the decode kernels store straight into the page-locked host buffer (no D2H copy)

    class _HostOut:
        ptr, nbytes = int(host.ctypes.data), host.nbytes
    if hostout:
        ref = ctx.alloc(T * T * 2)
        for bbox in qs[:20]:  # the host-resident result equals the device-resident one
            f = streaming.first_intersecting(index, bbox)
            i = f["frame_id"]
            n = f["window"]["width"] * f["window"]["height"]
            args = (arena, np.array([off[i], off[i + 1]], dtype=np.int64), [n])
            kw = dict(channels=1, bps=16, data_min=[float(mn[i])], data_max=[float(mx[i])], dtype=np.int16)
            ctx.decode_tiles_device(*args, out=ref, **kw)
            a = ref.download(n * 2).view(np.int16)
            ctx.decode_tiles_device(*args, out=_HostOut, **kw)
            assert np.array_equal(a, host[:n]), "host-resident decode differs"
        out = _HostOut
    ctx.profile(prof)
    ctx.profile_reset()
    for k, bbox in enumerate(qs[:10] + qs):
        t0 = time.perf_counter()
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"]
        n = f["window"]["width"] * f["window"]["height"]
        t1 = time.perf_counter()
        if old1:  # the round-5-before binding: per-call ctypes tables into frs_decode_tiles_device
            soff, poff, dmn, dmx = tabs
            soff[0], soff[1] = int(off[i]), int(off[i + 1])
            poff[1] = int(n)
            dmn[0], dmx[0] = float(mn[i]), float(mx[i])
            ctx._check(ctx.lib.frs_decode_tiles_device(ctx.handle, ctypes.c_void_p(arena.ptr), soff, 1, 1, 16, 4096,
                                                       poff, dmn, dmx, _native.DTYPE_CODES[np.dtype(np.int16)],
                                                       ctypes.c_void_p(out.ptr)))
        elif one:
            ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, mn[i], mx[i], np.int16, out)
        else:
            ctx.decode_tiles_device(arena, np.array([off[i], off[i + 1]], dtype=np.int64), [n], channels=1, bps=16,
                                    data_min=[float(mn[i])], data_max=[float(mx[i])], dtype=np.int16, out=out)
        t2 = time.perf_counter()
        if not hostout:
            out.download(n * 2, 0, out=host[:n].view(np.uint8))
        t3 = time.perf_counter()
        if k >= 10:
            ts.append(t1 - t0)
            td.append(t2 - t1)
            tc.append(t3 - t2)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("decode", "decode_span", "decode_frames")}
    p = lambda a: round(float(np.percentile(np.array(a) * 1e3, 50)), 4)
    tot = [a + b + c for a, b, c in zip(ts, td, tc)]
    print(json.dumps({"select_ms": p(ts), "decode_call_ms": p(td), "download_ms": p(tc), "total_p50": p(tot),
                      "total_p90": round(float(np.percentile(np.array(tot) * 1e3, 90)), 4),
                      "total_pct_10_25_75_95_99": [round(float(np.percentile(np.array(tot) * 1e3, q)), 4)
                                                   for q in (10, 25, 75, 95, 99)], "kernels": kern}))


if __name__ == "__main__":
    main()
