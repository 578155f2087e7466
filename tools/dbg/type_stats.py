"""debug: subframe type / LPC order / partition order histogram of the bench workload (C4 recipe, 2048 rows)"""
import sys
from collections import Counter
import numpy as np
sys.path.insert(0, ".")
from flac_raster_amd import _native
from oracle import oracle as O

ctx = _native.Context(0)
H, W, T, rows = 40000, 40000, 512, 2048
raster = ctx.alloc(4 * rows * W * 2)
ctx.synth_raster(raster, 4, rows, W, row0=0, full_height=H, seed=1234)
d = ctx.make_desc(rows, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100)
arena = ctx.alloc(rows * W * 3)
off, mn, mx, bps = ctx.encode_tiles_device(raster.ptr, d, arena)
blob = arena.download(int(off[-1]))
types, pos = Counter(), Counter()
for t in range(len(off) - 1):
    st = O.subframe_types(blob[off[t]:off[t + 1]].tobytes(), 1, 16, T * T)
    types.update(st[:, 0].tolist())
    pos.update(st[:, 1].tolist())
n = sum(types.values())
print("frames", n, "bytes/frame", off[-1] / n)
for k, v in sorted(types.items()):
    name = "CONST" if k == 0 else "VERB" if k == 1 else f"FIXED{k - 8}" if k < 32 else f"LPC{k - 31}"
    print(f"{name:8s} {v:7d} {v / n:.3f}")
print("partition orders", sorted(pos.items()))
