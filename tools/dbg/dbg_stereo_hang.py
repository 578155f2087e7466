"""Debug: one stereo case through the encoder with a Python traceback dump if it stalls (kernel names profiled)."""
import faulthandler
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
faulthandler.dump_traceback_later(40, exit=True)
import numpy as np  # noqa: E402
from flac_raster_amd import _native  # noqa: E402
from tests.test_gpu_stereo import _cases  # noqa: E402

case = int(sys.argv[1]) if len(sys.argv) > 1 else 6
name, arr, bits = _cases()[case]
B, H, W = arr.shape
ctx = _native.Context(0)
d = ctx.make_desc(H, W, arr.dtype, nbands=2, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=bits)
print("encoding", name, arr.shape, flush=True)
arena, off, mn, mx, bps = ctx.encode_tiles_host(arr, d)
print("done", len(arena), bps, flush=True)
