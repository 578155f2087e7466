#!/usr/bin/env python3
"""Per-wave timeline of the fused analysis kernel (k_analyze_v3<I16, false, true>) on C4, from an instrumented
variant library (timing only; never the product).

Build (CPU):   python tools/ana_timeline.py build      -> variants/libtl.so
Run (GPU box): FRS_LIB_PATH=variants/libtl.so python tools/ana_timeline.py run [out.npy]

Each wave records s_memrealtime (100 MHz) at its start, after its tile's min/max + LUT, and at its end, plus its
HW_ID / XCC_ID, into a device array read back through an extra export of the variant (frs_dbg_timeline).
The summary prints the stats and autocorrelation phase durations, the start-time spread, how many waves each SIMD
ran and the kernel's span, so the min/max bursts and the 1.5-round tail can be measured instead of guessed.
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

KERNEL_HEAD = "    const int2 wt = wtab[wv];  // (tile, first frame of the tile handled by this wave)\n"
STATS_END = "            if (lane == 0) norms[t] = tn;\n        }\n"
LUT_END = "            __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LUT stores have landed (each wave reads only its own)\n"
FINISH = "    if (!live) return;\n    out[f * P.nch + chn] = analysis_finish(acc, or_acc, n, P, ft);\n}\n"


def patch(src: str) -> str:
    decl = ("__device__ unsigned long long g_tl[16384][4];\n"
            "extern \"C\" int frs_dbg_timeline(void *host, size_t bytes) {\n"
            "    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tl), bytes, 0, hipMemcpyDeviceToHost);\n}\n")
    anchor = "template <int DT, bool SLOW, bool STATS = false>\n__global__ void __launch_bounds__(256) k_analyze_v3("
    assert anchor in src
    src = src.replace(anchor, decl + anchor, 1)
    assert KERNEL_HEAD in src and LUT_END in src and FINISH in src
    src = src.replace(KERNEL_HEAD, KERNEL_HEAD + "    const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();\n"
                      "    unsigned long long tl1 = tl0;\n", 1)
    src = src.replace(LUT_END, LUT_END + "            tl1 = __builtin_amdgcn_s_memrealtime();\n", 1)
    fin = ("    if constexpr (STATS) {\n"
           "        const unsigned long long tl2 = __builtin_amdgcn_s_memrealtime();\n"
           "        if (lane == 0 && wv < 16384) {\n"
           "            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);\n"
           "            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);\n"
           "            g_tl[wv][0] = tl0; g_tl[wv][1] = tl1; g_tl[wv][2] = tl2;\n"
           "            g_tl[wv][3] = (unsigned long long)hw | ((unsigned long long)xcc << 32);\n"
           "        }\n    }\n")
    return src.replace(FINISH, fin + FINISH, 1)


def run(out_path=None):
    from flac_raster_amd import _native
    lib = _native.load_library()
    fn = lib.frs_dbg_timeline
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    H = W = 40000
    T = 512
    ctx = _native.Context(0)
    raster = ctx.alloc(4 * H * W * 2)
    ctx.synth_raster(raster, 4, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    for _ in range(4):
        ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    buf = np.zeros((16384, 4), dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    n = ((H + T - 1) // T) * ((W + T - 1) // T)
    tl = buf[:n].astype(np.int64)
    if out_path:
        np.save(out_path, tl)
    summarize(tl)


def summarize(tl):
    t0 = tl[:, 0].min()
    s, m, e = (tl[:, 0] - t0) * 10e-3, (tl[:, 1] - t0) * 10e-3, (tl[:, 2] - t0) * 10e-3  # us
    hw, xcc = tl[:, 3] & 0xFFFFFFFF, tl[:, 3] >> 32
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    _, per_simd = np.unique(key, return_counts=True)
    pct = lambda a: " / ".join(f"{np.percentile(a, q):.1f}" for q in (5, 50, 95))
    print(f"waves {len(s)}  span {e.max():.1f} us  SIMDs {len(per_simd)}  waves per SIMD min/median/max "
          f"{per_simd.min()}/{int(np.median(per_simd))}/{per_simd.max()}")
    print(f"start p5/p50/p95 {pct(s)} us; stats+LUT phase {pct(m - s)} us; autocorr phase {pct(e - m)} us")
    first = s < np.percentile(s, 50) + 1
    print(f"first-round waves {first.sum()}: stats {pct((m - s)[first])}, autoc {pct((e - m)[first])}; "
          f"later waves: stats {pct((m - s)[~first])}, autoc {pct((e - m)[~first])}")
    edges = np.linspace(0, e.max(), 21)
    act = [int(((s <= x) & (e > x)).sum()) for x in edges[:-1]]
    inst = [int(((s <= x) & (m > x)).sum()) for x in edges[:-1]]
    print("time(us)  active  in-stats")
    for x, a, b in zip(edges[:-1], act, inst):
        print(f"{x:8.1f} {a:7d} {b:9d}")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        from build_variant import build_variant
        print(build_variant("tl", patch))
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else None)
