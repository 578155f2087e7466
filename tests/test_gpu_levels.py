"""Compression levels 0..8 on the GPU encoder: bytes equal the oracle's restatement of libFLAC's level table
(docs/sonos-pyflac.txt:6926-6934; parity UNPINNED for levels other than 5, see tests/test_levels.py).

Levels other than 5 run the generic kernels (k_analyze + k_encode_frames with EncodeParams.max_lpc / max_po; at 6..8
k_analyze_lpc_hi's per-window LPC candidates of the subdivide_tukey apodizations, LPC order up to 12 and partition
order 6; at 1 / 4 on two channels loose mid/side: a leader pass per group of frames, then the coding pass); the fast
kernels hard-code level 5's search and are not selected.  Covered: mono, two channels (independent at 0 / 3,
exhaustive mid/side at 2 / 5 / 6..8, loose at 1 / 4), three channels, a 32-bit stream, the spatial {-1, 0, 1} mode,
partial last frames, the file-level convert / convert --spatial paths, and the level range check.
"""
import numpy as np
import pytest

from flac_raster_amd import _native, geotiff
from flac_raster_amd.converter import RasterFLACConverter
from flac_raster_amd.spatial_encoder import SpatialFLACEncoder
from oracle import oracle as O
from oracle import pipeline as P
from tests.test_levels import _ok_levels, level_signal

pytestmark = pytest.mark.gpu


def _raster(ch, H, W, seed, dtype=np.int16, scale=1.0):
    x = level_signal(H * W, ch, seed).astype(np.float64) * scale
    return x.T.reshape(ch, H, W).astype(dtype)


CASES = [
    ("mono_i16_partial", 1, 130, 300, np.int16, 1.0, 16),   # 39000 px: partial last frame
    ("stereo_i16", 2, 128, 256, np.int16, 1.0, 16),
    ("rgb_u8", 3, 96, 200, np.uint8, 1 / 256.0, 16),
    ("mono_i32", 1, 100, 123, np.int32, 1000.0, 24),        # 32-bit stream
    ("stereo_u16", 2, 90, 111, np.uint16, 1.0, 16),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_levels_match_oracle(gpu_ctx, case):
    name, ch, H, W, dtype, scale, bits = CASES[case]
    arr = _raster(ch, H, W, 20 + case, dtype, scale)
    if dtype == np.uint8:
        arr = (arr.astype(np.int64) + 128).astype(np.uint8)
    elif dtype == np.uint16:
        arr = (arr.astype(np.int64) + 40000).astype(np.uint16)
    pcm, omn, omx, obps = O.normalize(arr.transpose(1, 2, 0).reshape(-1, ch))
    for lv in _ok_levels(ch):
        d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=ch, tile_h=H, tile_w=W, sample_rate=44100,
                              bits_per_sample=bits, compression_level=lv)
        arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
        assert bps == obps and (mn[0], mx[0]) == (omn, omx), (name, lv)
        assert arena[:off[-1]].tobytes() == O.encode_frames(pcm, obps, 44100, level=lv), (name, lv)


def test_levels_streaming_tiles_match_oracle(gpu_ctx):
    """Mono tiles (the create-streaming shape, 16-bit) with edge tiles at every level: per-tile oracle streams."""
    band = _raster(1, 700, 650, 31)[0]
    T = 256
    for lv in range(9):
        d = gpu_ctx.make_desc(700, 650, band.dtype, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16,
                              compression_level=lv)
        arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
        i = 0
        for r in range(0, 700, T):
            for c in range(0, 650, T):
                sub = np.ascontiguousarray(band[r:r + T, c:c + T])
                pcm, _, _, ob = O.normalize(sub.reshape(-1, 1))
                assert arena[off[i]:off[i + 1]].tobytes() == O.encode_frames(pcm, ob, 44100, level=lv), (lv, i)
                i += 1


def test_levels_spatial_mode_matches_oracle(gpu_ctx):
    arr = (_raster(2, 80, 100, 41) // 64).astype(np.int16)
    B, H, W = arr.shape
    pcm = O.normalize_spatial(np.ascontiguousarray(arr.reshape(B, -1).T))
    for lv in range(9):
        d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16,
                              norm_mode=1, compression_level=lv)
        arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
        assert bps == 32
        assert arena.tobytes() == O.encode_frames(pcm, 32, 44100, level=lv), lv


def test_level_files_match_oracle_pipeline(gpu_ctx, tmp_path):
    """`convert -c 0` / `-c 3` and `convert --spatial -c 3` through the product API against the oracle pipeline."""
    arr = _raster(1, 130, 300, 51)
    t = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    src = tmp_path / "one.tif"
    geotiff.write(src, arr, t, 32636)
    r = geotiff.read(src)
    conv = RasterFLACConverter(gpu_ctx)
    for lv in (0, 3, 7):
        out = tmp_path / f"one_c{lv}.flac"
        conv.tiff_to_flac(src, out, compression_level=lv)
        ref, _ = P.plain_convert(r.data, list(r.transform), r.crs_string, r.nodata, embed=True, level=lv)
        assert out.read_bytes() == ref, lv
        back = tmp_path / f"back{lv}.tif"
        conv.flac_to_tiff(out, back)
        assert np.array_equal(geotiff.read(back).data, arr)
    sp = tmp_path / "one_spatial.flac"
    SpatialFLACEncoder(64, gpu_ctx).encode_spatial_flac(src, sp, compression_level=3, date="2026-01-01",
                                                        gzip_mtime=0)
    assert sp.read_bytes() == P.raw_frames(r.data, list(r.transform), r.crs_string, 64, "2026-01-01", 0, level=3)


def test_level_range_checked_by_abi(gpu_ctx):
    arr = _raster(1, 64, 64, 61)
    for lv in (-1, 9):
        d = gpu_ctx.make_desc(64, 64, arr.dtype, tile_h=64, tile_w=64, sample_rate=44100, bits_per_sample=16,
                              compression_level=lv)
        with pytest.raises(_native.FrsError):
            gpu_ctx.encode_tiles_host(arr[0], d)


def test_high_levels_and_loose_stereo_long_streams(gpu_ctx):
    """Many frames per stream: level 8's nine windows per signal, and the loose mid/side schedule of levels 1 / 4
    over several four-frame groups (the leader pass), against the oracle."""
    n = 26 * 4096 + 777
    t = np.arange(n)
    rng = np.random.default_rng(8)
    L = 3000 * np.sin(t / 200.0) + rng.normal(0, 30, n)
    R = np.where((t // 4096) % 6 < 3, L + rng.normal(0, 2, n), rng.normal(0, 3000, n))
    x = np.clip(np.stack([L, R], axis=1), -32768, 32767).astype(np.int16)
    H, W = 1, n
    arr = np.ascontiguousarray(x.T.reshape(2, H, W))
    pcm, omn, omx, obps = O.normalize(x)
    for lv in (1, 4, 6, 8):
        d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=2, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16,
                              compression_level=lv)
        arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
        assert arena[:off[-1]].tobytes() == O.encode_frames(pcm, obps, 44100, level=lv), lv
