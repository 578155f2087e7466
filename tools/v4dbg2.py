import ctypes, os, sys, time, numpy as np
sys.path.insert(0, os.getcwd())
from flac_raster_amd import _native, geotiff
r = geotiff.read('tests/golden/sample_dem.tif')
band = np.ascontiguousarray(r.data[0])
lib = _native.load_library()
fn = lib.frs_dbg_v4; fn.restype = ctypes.c_int; fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
with _native.Context(0) as ctx:
    d = ctx.make_desc(512, 512, band.dtype, tile_h=256, tile_w=256, sample_rate=44100, bits_per_sample=16)
    t0 = time.time()
    try:
        arena, off, mn, mx, bps = ctx.encode_tiles_host(band, d)
        print('encode done', time.time() - t0, list(off), flush=True)
    except Exception as e:
        print('encode error', e, time.time() - t0, flush=True)
    buf = np.zeros((8192, 6), dtype=np.uint32)
    print('dbg rc', fn(buf.ctypes.data, buf.nbytes))
    used = buf[buf[:, 0] > 0]
    print('waves recorded', len(used), 'stats-role', int((used[:, 0] == 2).sum()), 'stats tiles', int(used[:, 1].sum()),
          'autoc tiles', int(used[:, 2].sum()), 'spins', int(used[:, 3].sum()), 'timeouts', int(used[:, 4].sum()), 'epochs', set(used[:, 5].tolist()))
