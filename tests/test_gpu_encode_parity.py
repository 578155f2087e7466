"""GPU encode parity: HIP frames must be byte-identical to the oracle / reference fixtures.

The oracle (oracle/flac_oracle.c) is pinned by tests/golden/sample_rgb.flac and sample_dem.flac
(see test_oracle_golden.py); here the product path (libflac_raster_amd.so through its C-ABI) is checked
against it on the same input bytes.
"""
import numpy as np
import pytest

from flac_raster_amd import geotiff
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _gpu_tiles(ctx, band, tile, sample_rate=44100):
    H, W = band.shape
    bps = 16 if band.dtype in (np.uint8, np.uint16, np.int16) else 24
    d = ctx.make_desc(H, W, band.dtype, tile_h=tile, tile_w=tile, sample_rate=sample_rate, bits_per_sample=bps)
    return ctx.encode_tiles_host(band, d)


def test_sample_rgb_plain_convert_bytes(gpu_ctx, golden):
    """converter.tiff_to_flac on sample_rgb.tif: 3 interleaved channels -> sample_rgb.flac frames."""
    r = geotiff.read(golden / "sample_rgb.tif")
    ref = (golden / "sample_rgb.flac").read_bytes()
    d = gpu_ctx.make_desc(256, 256, np.uint8, nbands=3, tile_h=256, tile_w=256, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(r.data, d)
    assert bps == 16 and mn[0] == 1.0 and mx[0] == 255.0
    assert arena.tobytes() == ref[86:]


def test_sample_rgb_band1_streaming_tile(gpu_ctx, golden):
    r = geotiff.read(golden / "sample_rgb.tif")
    band = np.ascontiguousarray(r.data[0])
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 512)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 512)
    assert arena.tobytes() == o_arena.tobytes()
    assert list(off) == list(o_off)
    assert list(mn) == list(o_mn) and list(mx) == list(o_mx)


def test_sample_dem_tiles_256(gpu_ctx, golden):
    r = geotiff.read(golden / "sample_dem.tif")
    band = np.ascontiguousarray(r.data[0])
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 256)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 256)
    assert list(off) == list(o_off)
    assert arena.tobytes() == o_arena.tobytes()


@pytest.mark.parametrize("dtype,shape,tile,seed", [
    (np.int16, (1100, 700), 512, 1),      # edge tiles, partial frames (700*76 px)
    (np.uint16, (600, 1030), 256, 2),
    (np.uint8, (300, 333), 128, 3),       # odd widths: frames span partial rows
    (np.int16, (64, 64), 512, 4),         # single 1-frame tile
])
def test_synthetic_tiles_match_oracle(gpu_ctx, dtype, shape, tile, seed):
    rng = np.random.default_rng(seed)
    H, W = shape
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    base = 1000 + 300 * np.sin(x * 0.8) * np.cos(y * 0.3) + 50 * rng.random((H, W))
    if dtype == np.uint8:
        base = base / 8
    band = base.astype(dtype)
    band[5:9, 5:40] = band[5, 5]  # a flat patch
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, tile)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile)
    assert list(off) == list(o_off)
    assert arena.tobytes() == o_arena.tobytes()


def test_constant_and_wasted_bits(gpu_ctx):
    band = np.full((128, 128), 7, dtype=np.int16)
    band[64:, :] = 9
    band[:, 100:] = 4000            # min/max spread so normalised samples have wasted bits in places
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 128)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 128)
    assert arena.tobytes() == o_arena.tobytes()


def test_full_range_int16_wraps_like_numpy(gpu_ctx):
    """Q2: x - min and max - min wrap in int16 (numpy 2); parity vs the oracle's restatement."""
    rng = np.random.default_rng(99)
    band = rng.integers(-32768, 32767, size=(256, 256), dtype=np.int16)
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 256)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 256)
    assert arena.tobytes() == o_arena.tobytes()


def test_int32_raster_32bit_stream(gpu_ctx):
    """bits_per_sample 24 -> pyflac itemsize 32-bit stream (Q4), limit_residual fixed estimator."""
    rng = np.random.default_rng(5)
    band = (rng.integers(0, 100000, size=(96, 200)) + np.arange(200) * 1000).astype(np.int32)
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 96)
    assert bps == 32
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 96)
    assert arena.tobytes() == o_arena.tobytes()


def test_decode_roundtrip_and_denormalize(gpu_ctx, golden):
    r = geotiff.read(golden / "sample_rgb.tif")
    ref = (golden / "sample_rgb.flac").read_bytes()
    frames = ref[86:]
    pcm = gpu_ctx.decode_frames_host(frames, [0, len(frames)], [65536], channels=3, bps=16)
    o_pcm = O.decode_frames(frames, 3, 16, 70000)
    assert np.array_equal(pcm, o_pcm)
    out = gpu_ctx.denormalize_host(pcm, 1.0, 255.0, np.uint8)
    assert np.array_equal(out, O.denormalize_i16(pcm, 1.0, 255.0, np.uint8))
    # lossless for uint8: back to the TIFF pixels
    assert np.array_equal(out.reshape(256, 256, 3).transpose(2, 0, 1), r.data)
    # fused decode + de-normalisation (3 interleaved channels: the wave decoder with the int32 scratch)
    fused = gpu_ctx.decode_tiles_host(frames, [0, len(frames)], [65536], channels=3, bps=16, data_min=[1.0],
                                      data_max=[255.0], dtype=np.uint8)
    assert np.array_equal(fused, out)


@pytest.mark.parametrize("dtype,lo,hi,shape,tile", [
    (np.int16, 900, 1800, (1024, 1536), 512),     # LUT normalisation (range < 4096)
    (np.uint16, 0, 40000, (512, 512), 256),       # exact reciprocal division (range 4096..65535)
    (np.int16, -30000, 30000, (512, 512), 512),   # wrapping int16 range (slow exact path)
    (np.uint8, 0, 255, (384, 640), 128),
    (np.uint16, 5, 6, (256, 256), 64),            # near-constant tiles: wasted bits / constant subframes
])
def test_fast_path_matches_oracle(gpu_ctx, dtype, lo, hi, shape, tile):
    rng = np.random.default_rng(hash((lo, hi)) % 1000)
    H, W = shape
    y, x = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    smooth = lo + (hi - lo) * (0.5 + 0.45 * np.sin(6 * x) * np.cos(4 * y))
    band = np.clip(smooth + rng.normal(0, (hi - lo) * 0.01 + 0.3, (H, W)), lo, hi).astype(dtype)
    band[:tile // 2, :tile // 2] = band[0, 0]        # a constant quarter tile
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, tile)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile)
    assert list(off) == list(o_off)
    assert arena.tobytes() == o_arena.tobytes()
    assert list(mn) == list(o_mn) and list(mx) == list(o_mx)


@pytest.mark.parametrize("kind,shape,tile", [
    ("noise", (1024, 1024), 512),     # VERBATIM-heavy frames (uniform full-range noise)
    ("dem", (2048, 3072), 512),       # 1536 frames: look-back spans many 64-frame windows, many tickets per WG
    ("dem", (512, 4096), 64),         # one frame per tile: a WG's 4 frames sit in 4 tiles
])
def test_fast_path_scale_and_noise(gpu_ctx, kind, shape, tile):
    rng = np.random.default_rng(4242)
    H, W = shape
    if kind == "noise":
        band = rng.integers(-32768, 32768, size=shape, dtype=np.int16)
    else:
        y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
        band = (1000 + 300 * np.sin(x * 0.8) * np.cos(y * 0.3) + 150 * np.sin(1.2 * x) * np.sin(1.1 * y)
                + 50 * rng.random(shape)).astype(np.int16)
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, tile)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile, threads=8)
    assert list(off) == list(o_off)
    assert arena.tobytes() == o_arena.tobytes()


@pytest.mark.parametrize("dtype,lo,hi,tile", [
    (np.int16, 900, 1800, 512),      # LUT tiles
    (np.uint16, 0, 40000, 256),      # fast-division tiles (the SLOW analysis launch)
    (np.int16, -30000, 30000, 128),  # wrapping range (exact division)
])
def test_fast_path_stats_modes(gpu_ctx, dtype, lo, hi, tile):
    """The fast path's tile stats run fused into the analysis launch (16-bit samples, 16-byte aligned rows, tiles
    of <= 64 frames) or as separate kernels before it (k_tile_stats(_vec) + k_tile_finalize + k_build_lut: tiles of
    more than 64 frames, rows that are not 16-byte runs).  Each geometry below takes one route -- checked through
    the per-kernel profile ("stats" is timed only when the separate kernels run) -- and both must give the
    oracle's bytes, also on a second call."""
    rng = np.random.default_rng(99)
    for H, W, t, fused in ((768, 1280, tile, True), (1100, 1300, 1024, False), (700, 1283, tile, False)):
        y, x = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
        band = np.clip(lo + (hi - lo) * (0.5 + 0.45 * np.sin(7 * x) * np.cos(3 * y))
                       + rng.normal(0, (hi - lo) * 0.01 + 0.3, (H, W)), lo, hi).astype(dtype)
        band[:t, :t] = band[0, 0]
        o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, t, threads=8)
        for _ in range(2):  # second call reuses the scratch
            gpu_ctx.profile(True)
            gpu_ctx.profile_reset()
            arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, t)
            gpu_ctx.profile(False)
            assert (gpu_ctx.profile_avg_ms("stats") <= 0) == fused, (H, W, t)
            assert list(off) == list(o_off), (H, W, t)
            assert arena.tobytes() == o_arena.tobytes(), (H, W, t)
            assert list(mn) == list(o_mn) and list(mx) == list(o_mx), (H, W, t)


@pytest.mark.parametrize("dtype,bands,shape,seed", [
    (np.uint8, 3, (300, 500), 1),       # sample_rgb-like, partial last frame
    (np.int16, 4, (1024, 1024), 2),     # whole frames only
    (np.uint16, 5, (640, 701), 3),
    (np.int16, 7, (256, 300), 4),
    (np.uint16, 8, (200, 333), 5),      # FLAC's channel limit: a 70 KB LDS frame image
])
def test_multichannel_fast_path_matches_oracle(gpu_ctx, dtype, bands, shape, seed):
    """Plain convert of a >= 3-band raster (converter.py:185-216: one stream, channels interleaved): the fast kernels
    code the subframes and k_mc_assemble joins them; bytes equal the oracle's libFLAC restatement."""
    H, W = shape
    rng = np.random.default_rng(seed)
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    data = np.stack([1000 + 300 * np.sin(x * (0.5 + 0.1 * b)) * np.cos(y * 0.3) + 40 * rng.random((H, W))
                     for b in range(bands)])
    if dtype == np.uint8:
        data = data / 8
    data = data.astype(dtype)
    data[:, 5:9, 5:40] = data[:, 5:6, 5:6]  # flat patches
    sr = O.sample_rate_for(bands, H)
    gpu_ctx.profile(True)
    gpu_ctx.profile_reset()
    d = gpu_ctx.make_desc(H, W, dtype, nbands=bands, tile_h=H, tile_w=W, sample_rate=sr, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(data, d)
    assembled = gpu_ctx.profile_avg_ms("assemble")
    gpu_ctx.profile(False)
    assert assembled > 0, "expected the multi-channel fast path"
    pcm, o_mn, o_mx, o_bps = O.normalize(data.transpose(1, 2, 0).reshape(-1, bands))
    ref = O.encode_frames(pcm, o_bps, sr)
    assert bps == o_bps == 16
    assert arena[:off[-1]].tobytes() == ref
    assert (mn[0], mx[0]) == (o_mn, o_mx)


def test_host_encode_batched_tile_ranges(gpu_ctx):
    """frs_encode_tiles on a large single band goes through the batched, overlapped upload path (tile-row batches,
    pinned ring, separate copy streams); a tile range that starts and ends mid-row must give the same bytes,
    offsets and min/max as the whole job's corresponding tiles, and the whole job must equal the oracle."""
    rng = np.random.default_rng(21)
    H, W, T = 6000, 6000, 512
    y, x = np.meshgrid(np.linspace(0, 20, H, dtype=np.float32), np.linspace(0, 20, W, dtype=np.float32),
                       indexing="ij")
    band = (1000 + 300 * np.sin(x * 0.8) * np.cos(y * 0.3) + 50 * rng.random((H, W), dtype=np.float32)).astype(np.int16)
    arena, off, mn, mx, _ = _gpu_tiles(gpu_ctx, band, T)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, T, threads=8)
    assert np.array_equal(off, o_off) and arena.tobytes() == o_arena.tobytes()
    d = gpu_ctx.make_desc(H, W, band.dtype, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16,
                          tile_begin=5, tile_end=131)
    a2, off2, mn2, mx2, _ = gpu_ctx.encode_tiles_host(band, d)
    assert np.array_equal(off2, off[5:132] - off[5])
    assert a2.tobytes() == arena[off[5]:off[131]].tobytes()
    assert np.array_equal(mn2, mn[5:131]) and np.array_equal(mx2, mx[5:131])


def test_geometry_cache_across_jobs(gpu_ctx):
    """The context caches the fast path's job geometry (tile table, partial list, wave table, frame -> tile map)
    while the descriptor repeats: jobs of alternating shapes, dtypes and tile sizes on one context -- each repeat
    hits the cache, each change rebuilds it -- must all equal the oracle."""
    rng = np.random.default_rng(11)
    jobs = [(np.int16, (1100, 700), 512), (np.int16, (1100, 700), 256), (np.uint16, (1100, 700), 512),
            (np.int16, (900, 1300), 512)]
    bands = [((rng.normal(0, 40, shape).cumsum(axis=1)) % 20000).astype(dt) for dt, shape, _ in jobs]
    refs = [O.encode_tiles(b, t)[0].tobytes() for b, (_, _, t) in zip(bands, jobs)]
    for i in (0, 0, 1, 1, 0, 2, 2, 0, 3, 3, 0):
        arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, bands[i], jobs[i][2])
        assert arena.tobytes() == refs[i], f"job {i}"


def test_many_small_tiles_match_oracle():
    """384 tiles of 128^2 (6 frames each) in one job, twice on one context (the geometry cache reused): bytes,
    offsets and min/max equal the oracle's (every look-back crosses many work-groups' tickets)."""
    from flac_raster_amd import _native
    rng = np.random.default_rng(21)
    band = (rng.normal(0, 30, (2048, 3072)).cumsum(axis=0) % 30000).astype(np.int16)  # 384 tiles of 128^2
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 128, threads=4)
    with _native.Context(0) as ctx:
        for _ in range(2):
            arena, off, mn, mx, bps = _gpu_tiles(ctx, band, 128)
            assert list(off) == list(o_off)
            assert arena.tobytes() == o_arena.tobytes()
            assert list(mn) == list(o_mn) and list(mx) == list(o_mx)


@pytest.mark.parametrize("kind", ["spikes", "burst", "steps16"])
def test_lane_segment_overflow_matches_oracle(gpu_ctx, kind):
    """The fast encoder packs each lane's 64 Rice codes into a private LDS column of 1088 bits; a lane whose codes
    outgrow it (a residual spike in a smooth frame: one code of thousands of unary bits) makes the wave repack the
    frame at its known offsets, and a lane whose segment is far longer than the frame's per-lane average spans
    three columns of the frame layout.  Frames of every kind must still be the oracle's bytes."""
    rng = np.random.default_rng(77)
    H = W = 512
    y, x = np.meshgrid(np.linspace(0, 6, H), np.linspace(0, 6, W), indexing="ij")
    band = (2000 + 900 * np.sin(x) * np.cos(y)).astype(np.int16)
    if kind == "spikes":      # isolated +-30000 samples: single huge codes
        band.flat[rng.choice(band.size, 60, replace=False)] = rng.choice([-30000, 30000], 60).astype(np.int16)
    elif kind == "burst":     # a 64-sample run of noise inside smooth frames: one lane's segment ~16 bits/sample
        for f in range(0, band.size // 4096, 3):
            s = f * 4096 + 64 * int(rng.integers(1, 63))
            band.flat[s:s + 64] = rng.integers(-32000, 32000, 64).astype(np.int16)
    else:                     # steps of exactly 16-bit residual magnitude on alternate lanes
        band.flat[::128] += 16000
    arena, off, mn, mx, bps = _gpu_tiles(gpu_ctx, band, 256)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, 256, threads=8)
    assert list(off) == list(o_off)
    assert arena.tobytes() == o_arena.tobytes()
