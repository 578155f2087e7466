"""BASELINE.json configs C3, C4 and C5 at full size on the HIP path, checked against the oracle.

C3: 16384^2 x 4 int16, tile 512 -- every tile's bytes, offsets and min/max equal the oracle's.
C4: 40000^2 x 4 int16, tile 512 (6241 tiles, 3.1 GB of frames) -- every tile byte-checked against the oracle
    (incl. the 64-px edge row 78 with the 64x64 corner tile), then every tile decoded in ONE fused decode call
    (a > 2 GiB range) and compared with the raster (the round trip is lossless).
C5: the 1000 seed-7 bbox queries on the C4 streaming data -- the grid-accelerated selection equals the linear scan
    of cli.py:976-987 and each decoded tile equals the oracle's decode + de-normalisation of the same bytes.
The rasters are generated on the device (frs_synth_raster_device) and downloaded, so the oracle sees the same
bytes as the GPU.
"""
import numpy as np
import pytest

import workloads
from oracle import oracle as O

pytestmark = pytest.mark.gpu

T = 512


def _device_raster(ctx, H, W, bands=4, seed=1234):
    raster = ctx.alloc(bands * H * W * 2)
    ctx.synth_raster(raster, bands, H, W, seed=seed)
    band = np.empty((H, W), dtype=np.int16)
    raster.download(H * W * 2, 0, out=band.view(np.uint8).reshape(-1))
    return raster, band


def _encode_device(ctx, raster, H, W):
    desc = ctx.make_desc(H, W, np.int16, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, bps = ctx.encode_tiles_device(raster.ptr, desc, arena)
    assert bps == 16
    return arena, off, mn, mx


def _check_tile_rows(band, arena, off, mn, mx, r0, r1, tcols):
    """Tile rows [r0, r1) of the GPU job against the oracle's encode of the same slab."""
    H, W = band.shape
    slab = np.ascontiguousarray(band[r0 * T:min(r1 * T, H)])
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(slab, T, threads=workloads.oracle_threads())
    t0, t1 = r0 * tcols, r1 * tcols
    got = arena.download(int(off[t1] - off[t0]), int(off[t0]))
    assert np.array_equal(np.diff(off[t0:t1 + 1]), np.diff(o_off)), f"tile sizes of rows {r0}..{r1}"
    assert got.tobytes() == o_arena.tobytes(), f"bytes of tile rows {r0}..{r1}"
    assert np.array_equal(mn[t0:t1], o_mn) and np.array_equal(mx[t0:t1], o_mx)


def _check_lossless(dec, band):
    """dec: tile-major decoded samples (row-major tiles, row-major pixels inside a tile) == band."""
    H, W = band.shape
    full, edge = W // T, W % T
    p = 0
    for r0 in range(0, H, T):
        h = min(T, H - r0)
        seg = dec[p:p + h * W]
        if full:
            blk = seg[:full * h * T].reshape(full, h, T).transpose(1, 0, 2).reshape(h, full * T)
            assert np.array_equal(blk, band[r0:r0 + h, :full * T]), f"tile row at {r0}"
        if edge:
            assert np.array_equal(seg[full * h * T:].reshape(h, edge), band[r0:r0 + h, full * T:]), f"edge at {r0}"
        p += h * W
    assert p == dec.size


# ----------------------------------------------------------------------------------------------------------- C3
def test_c3_full_raster_matches_oracle(gpu_ctx):
    H = W = 16384
    raster, band = _device_raster(gpu_ctx, H, W)
    arena, off, mn, mx = _encode_device(gpu_ctx, raster, H, W)
    assert len(off) == 32 * 32 + 1
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, T, threads=workloads.oracle_threads())
    assert np.array_equal(off, o_off)
    assert np.array_equal(mn, o_mn) and np.array_equal(mx, o_mx)
    got = arena.download(int(off[-1]), 0)
    assert got.tobytes() == o_arena.tobytes()
    # fused batched decode of all 1024 tiles, lossless
    counts = [T * T] * 1024
    out = gpu_ctx.alloc(H * W * 2)
    gpu_ctx.decode_tiles_device(arena, off, counts, channels=1, bps=16, data_min=mn, data_max=mx, dtype=np.int16,
                                out=out)
    dec = np.empty(H * W, dtype=np.int16)
    out.download(H * W * 2, 0, out=dec.view(np.uint8))
    _check_lossless(dec, band)
    for b in (out, arena, raster):
        b.close()


def test_c3_shape_full_range_noise_matches_oracle(gpu_ctx):
    """SURVEY 8d adversarial variant: uniform full-range int16 noise (seed 99) -- NEP 50 wrap of x - min, VERBATIM
    and high Rice parameters at scale (8192 x 8192, 256 tiles)."""
    H = W = 8192
    band = np.random.default_rng(99).integers(-32768, 32768, size=(H, W), dtype=np.int16)
    d = gpu_ctx.make_desc(H, W, np.int16, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, T, threads=workloads.oracle_threads())
    assert np.array_equal(off, o_off)
    assert arena.tobytes() == o_arena.tobytes()


# ----------------------------------------------------------------------------------------------------------- C4
@pytest.fixture(scope="module")
def c4(gpu_ctx):
    H = W = 40000
    raster, band = _device_raster(gpu_ctx, H, W)
    arena, off, mn, mx = _encode_device(gpu_ctx, raster, H, W)
    yield dict(H=H, W=W, raster=raster, band=band, arena=arena, off=off, mn=mn, mx=mx)
    arena.close()
    raster.close()


def test_c4_all_tiles_match_oracle(c4):
    """Every one of the 6241 C4 tiles (3.1 GB of frames): bytes, offsets and min/max equal the oracle's encode of
    the same raster, checked in slabs of 10 tile rows (host memory bounded); row 78 holds the 64-px-high edge tiles
    and the 64 x 64 corner tile."""
    tcols = (c4["W"] + T - 1) // T
    trows = (c4["H"] + T - 1) // T
    assert tcols == 79 and len(c4["off"]) == 79 * 79 + 1
    assert c4["off"][-1] > 2 ** 31  # the arena is larger than 2 GiB
    for r0 in range(0, trows, 10):
        _check_tile_rows(c4["band"], c4["arena"], c4["off"], c4["mn"], c4["mx"], r0, min(trows, r0 + 10), tcols)


def test_c4_decode_all_tiles_one_call_lossless(gpu_ctx, c4):
    from flac_raster_amd import streaming
    H, W = c4["H"], c4["W"]
    counts = [w * h for (_, _, w, h) in streaming.tile_grid(H, W, T)]
    out = gpu_ctx.alloc(H * W * 2)
    gpu_ctx.decode_tiles_device(c4["arena"], c4["off"], counts, channels=1, bps=16, data_min=c4["mn"],
                                data_max=c4["mx"], dtype=np.int16, out=out)
    dec = np.empty(H * W, dtype=np.int16)
    out.download(H * W * 2, 0, out=dec.view(np.uint8))
    out.close()
    _check_lossless(dec, c4["band"])


# ----------------------------------------------------------------------------------------------------------- C5
def test_c5_bbox_queries_match_linear_scan_and_oracle(gpu_ctx, c4):
    from flac_raster_amd import streaming
    H, W, off = c4["H"], c4["W"], c4["off"]
    index = workloads.streaming_index(H, W, T, np.diff(off))
    out = gpu_ctx.alloc(T * T * 2)
    host = np.empty(T * T, dtype=np.int16)
    for q, bbox in enumerate(workloads.c5_queries(H, W, T, 1000)):
        f = streaming.first_intersecting(index, bbox)
        hits = streaming.intersecting(index, bbox)
        assert hits and f is hits[0], q
        i = f["frame_id"]
        wnd = f["window"]
        n = wnd["width"] * wnd["height"]
        gpu_ctx.decode_tiles_device(c4["arena"], np.array([off[i], off[i + 1]], dtype=np.int64), [n], channels=1,
                                    bps=16, data_min=[c4["mn"][i]], data_max=[c4["mx"][i]], dtype=np.int16, out=out)
        out.download(n * 2, 0, out=host[:n].view(np.uint8))
        got = host[:n].reshape(wnd["height"], wnd["width"])
        frames = c4["arena"].download(int(off[i + 1] - off[i]), int(off[i])).tobytes()
        ref = O.denormalize_i16(O.decode_frames(frames, 1, 16, n), c4["mn"][i], c4["mx"][i], np.int16)
        assert np.array_equal(got.reshape(-1), ref.reshape(-1)), q
        r0, c0 = wnd["row_off"], wnd["col_off"]
        assert np.array_equal(got, c4["band"][r0:r0 + wnd["height"], c0:c0 + wnd["width"]]), q
    out.close()


def test_c5_host_resident_output(gpu_ctx, c4):
    """bench.py's C5 path: the fused decode stores each tile straight into page-locked host memory (frs_host_malloc,
    no D2H copy); results equal the raster windows, and a 3-channel stream (planar scratch + k_interleave_dn into
    host memory) equals the oracle."""
    from flac_raster_amd import streaming
    H, W, off = c4["H"], c4["W"], c4["off"]
    index = workloads.streaming_index(H, W, T, np.diff(off))
    hb = gpu_ctx.host_buffer(T * T * 2)
    host = hb.array.view(np.int16)
    for q, bbox in enumerate(workloads.c5_queries(H, W, T, 200)):
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"]
        wnd = f["window"]
        n = wnd["width"] * wnd["height"]
        host[:n] = -1
        gpu_ctx.decode_tile_device(c4["arena"], off[i], off[i + 1], n, 1, 16, c4["mn"][i], c4["mx"][i], np.int16, hb)
        r0, c0 = wnd["row_off"], wnd["col_off"]
        got = host[:n].reshape(wnd["height"], wnd["width"])
        assert np.array_equal(got, c4["band"][r0:r0 + wnd["height"], c0:c0 + wnd["width"]]), q
    hb.close()
    rng = np.random.default_rng(3)
    data = (1000 + 300 * np.sin(np.arange(3 * 300 * 400) / 50.0).reshape(3, 300, 400)
            + rng.integers(0, 40, (3, 300, 400))).astype(np.int16)
    d = gpu_ctx.make_desc(300, 400, np.int16, nbands=3, tile_h=300, tile_w=400, sample_rate=O.sample_rate_for(3, 300),
                          bits_per_sample=16)
    arena, toff, mn, mx, bps = gpu_ctx.encode_tiles_host(data, d)
    arena = np.ascontiguousarray(arena[:toff[-1]])
    blob = gpu_ctx.alloc(len(arena))
    blob.upload(arena)
    hb = gpu_ctx.host_buffer(data.nbytes)
    gpu_ctx.decode_tiles_device(blob, np.array([0, len(arena)], dtype=np.int64), [300 * 400], channels=3, bps=16,
                                data_min=[mn[0]], data_max=[mx[0]], dtype=np.int16, out=hb)
    pcm = O.decode_frames(arena.tobytes(), 3, 16, 300 * 400)
    ref = O.denormalize_i16(pcm, mn[0], mx[0], np.int16)
    assert np.array_equal(hb.array.view(np.int16).reshape(-1), ref.reshape(-1))
    hb.close()
    blob.close()


# ------------------------------------------------------------------------- partial frames on the fast path
@pytest.mark.parametrize("shape,tile,dtype", [
    ((10980, 10980), 1024, np.uint16),  # the reference's Sentinel-2 B04 example (FLAC-SPATIAL.md:82-88): last tile 740^2
    ((512, 512), 200, np.int16),        # sample_dem at tile 200: every tile ends in a partial frame
    ((1000, 1000), 30, np.int16),       # tiles smaller than one frame (900 px: a single partial frame each)
    ((1030, 4098), 128, np.int16),      # rows only 4-byte aligned (8196-B stride): dword chunk loads
])
def test_partial_frame_tiles_take_the_fast_path(gpu_ctx, shape, tile, dtype):
    """Tiles whose pixel count is not a multiple of 4096 keep the fast kernels (their partial last frames are coded
    by the generic kernels and joined into the fast encoder's look-back chain); bytes equal the oracle's."""
    H, W = shape
    rng = np.random.default_rng(11)
    y = np.linspace(0, 20, H, dtype=np.float32)[:, None]
    x = np.linspace(0, 20, W, dtype=np.float32)[None, :]
    base = 3000 + 1200 * np.sin(x * 0.7) * np.cos(y * 0.3) + 400 * np.sin(1.3 * x) * np.sin(1.1 * y)
    band = (base + 60 * rng.random((H, W), dtype=np.float32)).astype(dtype)
    gpu_ctx.profile(True)
    gpu_ctx.profile_reset()
    d = gpu_ctx.make_desc(H, W, dtype, tile_h=tile, tile_w=tile, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
    partial_ms, compact_ms = gpu_ctx.profile_avg_ms("partial"), gpu_ctx.profile_avg_ms("compact")
    gpu_ctx.profile(False)
    assert partial_ms > 0 and compact_ms < 0, "expected the fast path with a partial-frame pass"
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile, threads=workloads.oracle_threads())
    assert np.array_equal(off, o_off)
    assert arena.tobytes() == o_arena.tobytes()
    assert np.array_equal(mn, o_mn) and np.array_equal(mx, o_mx)


@pytest.mark.parametrize("shape,tile", [((4096, 6000), 512), ((3000, 3100), 1024), ((700, 900), 200)])
def test_prefetch_analysis_equals_plain_form(gpu_ctx, monkeypatch, shape, tile):
    """k_analyze_v3's prefetching launch (small jobs: the next chunk's loads in flight while one is summed) and the
    plain launch give the same frames, both equal to the oracle (fused stats at tile 512; separate stats and partial
    last frames at 1024 and 200)."""
    H, W = shape
    raster, band = _device_raster(gpu_ctx, H, W, bands=1, seed=77)
    outs = []
    for force in ("1", "0"):
        monkeypatch.setenv("FRS_ANA_PF", force)
        desc = gpu_ctx.make_desc(H, W, np.int16, tile_h=tile, tile_w=tile, sample_rate=44100, bits_per_sample=16)
        arena = gpu_ctx.alloc(gpu_ctx.arena_bound(desc))
        off, mn, mx, _ = gpu_ctx.encode_tiles_device(raster.ptr, desc, arena)
        outs.append((off.copy(), arena.download(int(off[-1]), 0).tobytes()))
        arena.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    o_arena, o_off, _, _ = O.encode_tiles(band, tile, threads=workloads.oracle_threads())
    assert np.array_equal(outs[0][0], o_off) and outs[0][1] == o_arena.tobytes()
    raster.close()
