import os, sys, time, numpy as np
sys.path.insert(0, os.getcwd())
from flac_raster_amd import _native, geotiff
from oracle import oracle as O
r = geotiff.read('tests/golden/sample_dem.tif')
band = np.ascontiguousarray(r.data[0])
print('dtype', band.dtype, band.shape, flush=True)
ref = O.encode_tiles(band, 256)
with _native.Context(0) as ctx:
    d = ctx.make_desc(512, 512, band.dtype, tile_h=256, tile_w=256, sample_rate=44100, bits_per_sample=16)
    t0 = time.time()
    arena, off, mn, mx, bps = ctx.encode_tiles_host(band, d)
    print('encode done', time.time() - t0, 'equal', arena.tobytes() == ref[0].tobytes(), list(off), list(ref[1]), flush=True)
    print('mn', list(mn), list(ref[2]), flush=True)
