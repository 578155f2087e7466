"""Raw-frames tiles (`convert --spatial`, spatial_encoder.py:186-193, 229-294) on the GPU against the oracle, tile by
tile: the spatial normalisation gives pyflac's truncated floats, so a DEM's subframes are almost all zero
(reference quirk Q1).  Round 6 codes all-zero subframes and frames on a fast path (k_zero_subframes,
k_zero_frames_emit); these cases mix all-zero subframes with {-1, 0, 1} ones inside the same frame and tile, cover
partial last frames (including one of 4 samples, which keeps the generic path), 1 and 3 bands, and int16 / uint8 /
uint16 rasters, so every byte of both paths is checked."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _raster(B, H, W, dtype, seed):
    rng = np.random.default_rng(seed)
    if dtype == np.int16:
        a = rng.integers(-3000, 3000, size=(B, H, W)).astype(np.int16)  # -> 0
        lo, hi = np.int16(-32768), np.int16(32767)                      # -> -1, 1
    elif dtype == np.uint8:
        a = rng.integers(1, 255, size=(B, H, W)).astype(np.uint8)
        lo, hi = np.uint8(0), np.uint8(255)
    else:
        a = rng.integers(1, 65535, size=(B, H, W)).astype(np.uint16)
        lo, hi = np.uint16(0), np.uint16(65535)
    # extremes in the top-left quarter only (the far tiles stay all-zero): rows of the last band (mixed zero /
    # non-zero subframes in one frame) and a sparse sprinkle in band 0 (frames with a few +-1 among zeros)
    a[-1, 5:9, :W // 2] = hi
    a[-1, 30:32, 10:W // 2] = lo
    m = rng.random((H // 3, W // 3)) < 0.01
    a[0, :H // 3, :W // 3][m] = hi
    return a


CASES = [
    ("i16_3band_tile128", np.int16, 3, 300, 400, 128, 128),
    ("i16_1band_n4", np.int16, 1, 82, 200, 41, 100),   # 4100-px tiles: a 4-sample last frame
    ("u8_3band_tile256", np.uint8, 3, 256, 300, 256, 256),
    ("u16_1band_tile64", np.uint16, 1, 200, 190, 64, 64),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_raw_frame_tiles_match_oracle(gpu_ctx, case):
    name, dtype, B, H, W, th, tw = CASES[case]
    arr = _raster(B, H, W, dtype, 50 + case)
    d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=B, tile_h=th, tile_w=tw, sample_rate=44100, bits_per_sample=16,
                          norm_mode=1)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
    assert bps == 32
    i = 0
    zero_only = mixed = 0
    for r in range(0, H, th):
        for c in range(0, W, tw):
            sub = np.ascontiguousarray(arr[:, r:r + th, c:c + tw])
            pcm = O.normalize_spatial(np.ascontiguousarray(sub.reshape(B, -1).T))
            ref = O.encode_frames(pcm, 32, 44100)
            assert arena[off[i]:off[i + 1]].tobytes() == ref, (name, i)
            if not pcm.any():
                zero_only += 1
            else:
                mixed += 1
            i += 1
    assert i == len(off) - 1
    assert zero_only and mixed, (zero_only, mixed)  # both kinds of tile occur
