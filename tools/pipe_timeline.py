#!/usr/bin/env python3
"""Per-frame timeline of the C5 latency decoder (k_decode_frames_pipe) from an instrumented variant library
(timing only; never the product).

Build (CPU):   python tools/pipe_timeline.py build     -> variants/libptl.so
Run (GPU box): FRS_LIB_PATH=variants/libptl.so python tools/pipe_timeline.py run

Each work-group (frame) records s_memrealtime (100 MHz) at its start, after staging the frame's words, when the
producer wave (parse + Rice decode) finishes, when the consumer wave (LPC restore) finishes its recurrence, and at
the consumer's end (samples stored), for 200 C5 queries' tiles; the summary prints the phase medians.
"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

HEAD = "    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;\n    const int64_t ci = frame_cand[fi];\n"
STAGED = "    if (threadIdx.x == 0) {\n        info.state = 0;\n"
PROD_END = ("        if (lane == 0) {\n            info.valid = ok;\n            lds_publish(&vi->progress, bad ? -1 : bs);\n"
            "            lds_publish(&vi->finished, 1);\n        }\n        return;\n    }\n")
CONS_REST = "    if (!failed && (bs & 1)) xout[bs >> 1] = H[0] & 0xFFFFu;\n"
CONS_END = "    if (lane == 0) atomicAdd(nvalid, 1);\n}\n\n// One wave per frame"


def patch(src: str) -> str:
    decl = ("__device__ unsigned long long g_ptl[1024][6];\n"
            "extern \"C\" int frs_dbg_pipe_timeline(void *host, size_t bytes) {\n"
            "    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptl), bytes, 0, hipMemcpyDeviceToHost);\n}\n")
    anchor = "__global__ void __launch_bounds__(128) k_decode_frames_pipe("
    for a in (anchor, HEAD, STAGED, PROD_END, CONS_REST, CONS_END):
        assert src.count(a) >= 1, a[:60]
    src = src.replace(anchor, decl + anchor, 1)
    src = src.replace(HEAD, HEAD + "    const unsigned long long tp0 = __builtin_amdgcn_s_memrealtime();\n"
                      "    const int fslot = (int)(fi & 1023);\n", 1)
    src = src.replace(STAGED, "    if (threadIdx.x == 0) { g_ptl[fslot][0] = tp0; g_ptl[fslot][1] = "
                      "__builtin_amdgcn_s_memrealtime(); }\n" + STAGED, 1)
    src = src.replace(PROD_END, PROD_END.replace("            lds_publish(&vi->finished, 1);\n",
                      "            lds_publish(&vi->finished, 1);\n            g_ptl[fslot][2] = "
                      "__builtin_amdgcn_s_memrealtime();\n"), 1)
    src = src.replace(CONS_REST, CONS_REST + "    if (lane == 0) g_ptl[fslot][3] = __builtin_amdgcn_s_memrealtime();\n", 1)
    src = src.replace(CONS_END, "    if (lane == 0) { g_ptl[fslot][4] = __builtin_amdgcn_s_memrealtime(); "
                      "g_ptl[fslot][5] = 1; }\n" + CONS_END, 1)
    return src


def run():
    import workloads
    from flac_raster_amd import _native, streaming
    lib = _native.load_library()
    fn = lib.frs_dbg_pipe_timeline
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
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
    out = ctx.alloc(T * T * 2)
    rows = []
    for bbox in workloads.c5_queries(H, W, T, 200):
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"]
        n = f["window"]["width"] * f["window"]["height"]
        ctx.decode_tiles_device(arena, np.array([off[i], off[i + 1]], dtype=np.int64), [n], channels=1, bps=16,
                                data_min=[float(mn[i])], data_max=[float(mx[i])], dtype=np.int16, out=out)
        ctx.sync()
        buf = np.zeros((1024, 6), dtype=np.uint64)
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        nf = (n + 4095) // 4096
        tl = buf[:nf].astype(np.int64)
        if (tl[:, 5] == 1).all():
            t0 = tl[:, 0].min()
            rows.append(((tl[:, :5] - t0) * 10e-3, (tl[:, 4].max() - t0) * 10e-3))
    ph = np.concatenate([r[0] for r in rows])
    med = lambda a: f"{np.percentile(a, 50):.1f} (p90 {np.percentile(a, 90):.1f})"
    print(f"tiles {len(rows)} frames {len(ph)}: kernel span (first start -> last end) {med([r[1] for r in rows])} us")
    print(f"start offset {med(ph[:, 0])}; staging {med(ph[:, 1] - ph[:, 0])}; producer (parse + Rice) "
          f"{med(ph[:, 2] - ph[:, 1])}; consumer restore done at {med(ph[:, 3] - ph[:, 1])}; stores "
          f"{med(ph[:, 4] - ph[:, 3])}; frame total {med(ph[:, 4] - ph[:, 0])} us")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        from build_variant import build_variant
        print(build_variant("ptl", patch, src_name="frs_decode.hip"))
    else:
        run()
