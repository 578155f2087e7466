"""Two-channel streams: libFLAC level 5's exhaustive mid/side stereo (do_mid_side_stereo = true,
loose_mid_side_stereo = false, docs/sonos-pyflac.txt:6931; assignments :2571-2576).

A 2-band `convert` (converter.py:185-216) or `convert --spatial` (spatial_encoder.py:186-193) hands pyflac a
[N, 2] array, so libFLAC codes left, right, mid and side every frame and writes the cheapest assignment.  The
HIP encoder must write the oracle's bytes, and the lane (k_decode_frames_lane + k_interleave_dn) and wave
(decode_one_frame) decoders must return the oracle's samples, for all four assignments, 16-bit streams (17-bit
side), 32-bit streams (33-bit side) and partial last frames.

Parity of the oracle itself is UNPINNED for two channels: no fixture of the reference holds a 2-channel stream;
the oracle restates stream_encoder.c process_subframes_ (see oracle/flac_oracle.c orc_encode_frames).
"""
import numpy as np
import pytest

from flac_raster_amd import geotiff
from flac_raster_amd.converter import RasterFLACConverter
from flac_raster_amd.spatial_encoder import SpatialFLACEncoder
from oracle import oracle as O
from oracle import pipeline as P

pytestmark = pytest.mark.gpu


def stereo_raster(H, W, seed, dtype=np.int16, scale=1.0, offset=2000.0):
    """Two bands whose 4096-sample frames cycle through independent / left-side / right-side / mid-side winners."""
    rng = np.random.default_rng(seed)
    n = H * W
    t = np.arange(n)
    base = 800 * np.sin(t / 300.0) + 200 * np.sin(t / 37.0)
    L, R = base.copy(), base.copy()
    for f in range((n + 4095) // 4096):
        sl = slice(f * 4096, min(n, (f + 1) * 4096))
        m = sl.stop - sl.start
        k = f % 4
        if k == 0:
            R[sl] = 600 * np.sin(t[sl] / 11.0 + f) + rng.normal(0, 30, m)
            L[sl] += rng.normal(0, 2, m)
        elif k == 1:
            R[sl] = L[sl] + rng.normal(0, 40, m)
        elif k == 2:
            L[sl] = R[sl] + rng.normal(0, 40, m)
        else:
            e = rng.normal(0, 20, m)
            L[sl] += e
            R[sl] -= e
    arr = (np.stack([L, R]).reshape(2, H, W) + offset) * scale
    return arr.astype(dtype)


def _cases():
    rgb = geotiff.read(__import__("pathlib").Path(__file__).parent / "golden" / "sample_rgb.tif").data
    rng = np.random.default_rng(11)
    eq = stereo_raster(96, 100, 3)
    eq[1] = eq[0]                                                   # side == 0: CONSTANT side subframes
    neg = stereo_raster(128, 96, 4)
    neg[1] = (4000 - neg[0]).astype(np.int16)
    return [
        ("i16_partial", stereo_raster(130, 300, 5, np.int16), 16),           # 39000 px: partial last frame
        ("u16", stereo_raster(200, 205, 6, np.uint16, 8.0), 16),
        ("u8", stereo_raster(130, 300, 7, np.float64, 1 / 16.0, 3000).astype(np.uint8), 16),
        ("rgb01", np.ascontiguousarray(rgb[:2]), 16),
        ("equal", eq, 16),
        ("negated", neg, 16),
        ("noise_i16", rng.integers(-32768, 32767, size=(2, 64, 200), dtype=np.int16), 16),
        ("i32", stereo_raster(100, 123, 8, np.int32, 1000.0), 24),           # 32-bit stream, 33-bit side
        ("f32_wide", _wide_float(64, 128, 9), 24),                            # |side| > 2^31
    ]


def _wide_float(H, W, seed):
    """float32 bands used as-is (converter.py:61-64, * 8388607): L ~ -R near +-140, so side = L - R needs 33 bits."""
    rng = np.random.default_rng(seed)
    t = np.arange(H * W)
    L = 140 * np.sin(t / 50.0) + rng.normal(0, 0.01, t.size)
    R = -0.99 * L + rng.normal(0, 0.01, t.size)
    return np.stack([L, R]).reshape(2, H, W).astype(np.float32)


def _oracle_frames(arr, bits):
    B, H, W = arr.shape
    pcm, mn, mx, bps = O.normalize(arr.transpose(1, 2, 0).reshape(-1, B))
    return O.encode_frames(pcm, bps, 44100), pcm, bps, mn, mx


@pytest.mark.parametrize("case", range(9))
def test_stereo_encode_matches_oracle(gpu_ctx, case):
    name, arr, bits = _cases()[case]
    B, H, W = arr.shape
    d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=2, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=bits)
    gpu_ctx.profile(True)
    gpu_ctx.profile_reset()
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
    compact_ms = gpu_ctx.profile_avg_ms("compact")
    gpu_ctx.profile(False)
    fr, pcm, obps, omn, omx = _oracle_frames(arr, bits)
    assert bps == obps and mn[0] == omn and mx[0] == omx, name
    assert arena.tobytes() == fr, name
    if bps == 16:  # 16-bit streams take the fast two-channel kernels (L, R, M as packed pairs, S as int32)
        assert compact_ms < 0, f"{name}: expected the fast stereo path, got the generic kernels"


def test_stereo_spatial_encode_matches_oracle(gpu_ctx):
    """2-band raw frames: float32 normalisation -> {-1, 0, 1} int32 samples, 32-bit stream, 33-bit side."""
    arr = stereo_raster(100, 90, 12, np.float64, 1 / 16.0, 3000).astype(np.uint8)
    arr[1, :, ::3] = 255 - arr[1, :, ::3]
    B, H, W = arr.shape
    d = gpu_ctx.make_desc(H, W, arr.dtype, nbands=2, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16,
                          norm_mode=1)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(arr, d)
    pcm = O.normalize_spatial(np.ascontiguousarray(arr.reshape(2, -1).T))
    assert bps == 32
    assert arena.tobytes() == O.encode_frames(pcm, 32, 44100)


def test_stereo_files_match_oracle_pipeline(gpu_ctx, tmp_path):
    """Whole files through the product API: 2-band convert (mutagen tags) and 2-band convert --spatial."""
    arr = stereo_raster(130, 300, 13, np.int16)
    t = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    src = tmp_path / "two.tif"
    geotiff.write(src, arr, t, 32636)
    r = geotiff.read(src)
    out = tmp_path / "two.flac"
    RasterFLACConverter(gpu_ctx).tiff_to_flac(src, out)
    ref, _ = P.plain_convert(r.data, list(r.transform), r.crs_string, r.nodata, embed=True)
    assert out.read_bytes() == ref
    sp = tmp_path / "two_spatial.flac"
    SpatialFLACEncoder(64, gpu_ctx).encode_spatial_flac(src, sp, date="2026-01-01", gzip_mtime=0)
    assert sp.read_bytes() == P.raw_frames(r.data, list(r.transform), r.crs_string, 64, "2026-01-01", 0)
    back = tmp_path / "back.tif"
    RasterFLACConverter(gpu_ctx).flac_to_tiff(out, back)
    assert np.array_equal(geotiff.read(back).data, arr)


DECODERS = {"lane": {"FRS_DECODE_LANE": "1"},      # lane-per-frame subframes -> planar -> k_interleave_dn
            "wave": {"FRS_FORCE_GENERIC": "1"}}    # one-lane wave decoder (decode_one_frame)


@pytest.mark.parametrize("kind", list(DECODERS))
def test_stereo_decode_matches_oracle(gpu_ctx, kind, monkeypatch):
    from flac_raster_amd import _native
    for k, v in DECODERS[kind].items():
        monkeypatch.setenv(k, v)
    dctx = _native.Context(0)
    # >= 64 frames so the lane decoder takes the job; every assignment; partial last frame
    cases = [("big", stereo_raster(515, 520, 21, np.int16), 16)] + _cases()
    for name, arr, bits in cases:
        fr, pcm, bps, mn, mx = _oracle_frames(arr, bits)
        n = pcm.shape[0]
        got = dctx.decode_frames_host(np.frombuffer(fr, np.uint8), [0, len(fr)], [n], channels=2, bps=bps)
        assert np.array_equal(got, pcm), (kind, name)
        if bps == 16:
            vals = dctx.decode_tiles_host(np.frombuffer(fr, np.uint8), [0, len(fr)], [n], channels=2, bps=16,
                                          data_min=[mn], data_max=[mx], dtype=arr.dtype)
            ref = O.denormalize_i16(pcm, mn, mx, arr.dtype)
            assert np.array_equal(vals, ref), (kind, name)
    dctx.close()
