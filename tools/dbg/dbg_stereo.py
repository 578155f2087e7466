"""debug: frame-by-frame comparison of the GPU two/three-channel encode with the oracle (noise rasters)"""
import sys
import numpy as np
sys.path.insert(0, ".")
from flac_raster_amd import _native
from oracle import oracle as O


def frames(b):
    out, i = [], 0
    idx = [j for j in range(len(b) - 1) if b[j] == 0xFF and b[j + 1] == 0xF8]
    return idx


def run(ctx, arr, bits=16):
    B, H, W = arr.shape
    d = ctx.make_desc(H, W, arr.dtype, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=bits)
    arena, off, mn, mx, bps = ctx.encode_tiles_host(arr, d)
    got = arena.tobytes()
    pcm, mn, mx, bps = O.normalize(arr.transpose(1, 2, 0).reshape(-1, B))
    exp = O.encode_frames(pcm, bps, 44100)
    print("B", B, "len got", len(got), "exp", len(exp), "equal", got == exp)
    if got != exp:
        k = next(i for i in range(min(len(got), len(exp))) if got[i] != exp[i])
        print("first diff", k)
        print("got", got[k - 12:k + 12].hex())
        print("exp", exp[k - 12:k + 12].hex())
        fe = [j for j in frames(exp) if exp[j + 2] == 0xC9]
        print("exp frame starts", fe[:8])


ctx = _native.Context(0)
rng = np.random.default_rng(11)
run(ctx, rng.integers(-32768, 32767, size=(2, 64, 200), dtype=np.int16))
rng = np.random.default_rng(11)
run(ctx, rng.integers(-32768, 32767, size=(3, 64, 200), dtype=np.int16))
rng = np.random.default_rng(12)
run(ctx, rng.integers(-32768, 32767, size=(2, 64, 256), dtype=np.int16))
run(ctx, rng.integers(-16384, 16383, size=(2, 64, 256), dtype=np.int16))
ctx.close()
