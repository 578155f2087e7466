"""Whole-file parity on the GPU: the product API writes the same bytes as the reference (fixtures) or
the oracle pipeline (its whole-file restatement, pinned by the fixtures in test_oracle_golden.py)."""
import base64
import struct

import numpy as np
import pytest

from flac_raster_amd import container, geotiff, streaming
from flac_raster_amd.converter import RasterFLACConverter
from flac_raster_amd.spatial_encoder import SpatialFLACEncoder
from oracle import pipeline as P

pytestmark = pytest.mark.gpu


def test_convert_sample_rgb_without_mutagen_is_fixture(gpu_ctx, golden, tmp_path):
    out = tmp_path / "rgb.flac"
    RasterFLACConverter(gpu_ctx, embed_metadata=False).tiff_to_flac(golden / "sample_rgb.tif", out)
    assert out.read_bytes() == (golden / "sample_rgb.flac").read_bytes()
    assert out.with_suffix(".json").read_text() == (golden / "sample_rgb.json").read_text()


def test_convert_with_mutagen_tags_matches_oracle(gpu_ctx, golden, tmp_path):
    for name in ("sample_rgb", "sample_multispectral", "sample_dem"):
        out = tmp_path / f"{name}.flac"
        RasterFLACConverter(gpu_ctx).tiff_to_flac(golden / f"{name}.tif", out)
        r = geotiff.read(golden / f"{name}.tif")
        ref, _ = P.plain_convert(r.data, list(r.transform), r.crs_string, r.nodata, embed=True)
        assert out.read_bytes() == ref, name


def test_flac_to_tiff_reconstructs_fixture(gpu_ctx, golden, tmp_path):
    src = tmp_path / "sample_rgb.flac"
    src.write_bytes((golden / "sample_rgb.flac").read_bytes())
    src.with_suffix(".json").write_text((golden / "sample_rgb.json").read_text())
    out = tmp_path / "rec.tif"
    RasterFLACConverter(gpu_ctx).flac_to_tiff(src, out)
    rec = geotiff.read(out)
    ref = geotiff.read(golden / "sample_rgb_reconstructed.tif")
    assert np.array_equal(rec.data, ref.data)
    assert rec.transform.to_tuple() == ref.transform.to_tuple() and rec.epsg == 4326


@pytest.mark.parametrize("name,tile", [("sample_rgb", 512), ("sample_rgb", 100), ("sample_dem", 256),
                                       ("sample_dem", 200), ("sample_multispectral", 64)])
def test_create_streaming_matches_oracle(gpu_ctx, golden, tmp_path, name, tile):
    out = tmp_path / f"{name}_{tile}.flac"
    streaming.create_streaming(golden / f"{name}.tif", out, tile, ctx=gpu_ctx)
    r = geotiff.read(golden / f"{name}.tif")
    ref = P.create_streaming(r.data[0], list(r.transform), r.crs_string, tile)
    assert out.read_bytes() == ref


def test_streaming_c2_tile_frames_are_fixture_channel0(gpu_ctx, golden, tmp_path):
    """C2: the single 256x256 band-1 tile's subframes equal channel 0 of sample_rgb.flac (band 1 has the
    global min/max 1..255, so the normalised samples are identical)."""
    from oracle import oracle as O
    out = tmp_path / "c2.flac"
    streaming.create_streaming(golden / "sample_rgb.tif", out, 512, ctx=gpu_ctx)
    n, index = streaming.read_index(out)
    tile = streaming.fetch_tiles(out, index["frames"], n)[0]
    m = container.parse_metadata(tile)
    pcm_tile = O.decode_frames(tile[m.audio_offset:], 1, 16, 70000)
    fx = (golden / "sample_rgb.flac").read_bytes()
    pcm_fx = O.decode_frames(fx[86:], 3, 16, 70000)
    assert np.array_equal(pcm_tile[:, 0], pcm_fx[:, 0])


def test_extract_streaming_roundtrip_lossless(gpu_ctx, golden, tmp_path):
    out = tmp_path / "dem.flac"
    streaming.create_streaming(golden / "sample_dem.tif", out, 200, ctx=gpu_ctx)
    r = geotiff.read(golden / "sample_dem.tif")
    n, index = streaming.read_index(out)
    for sel in (dict(tile_id=4), dict(last=True), dict(center=True), dict(bbox=[-105.3, 40.2, -105.25, 40.25])):
        tif = tmp_path / "t.tif"
        f = streaming.extract_streaming(out, tif, ctx=gpu_ctx, **sel)
        w = f["window"]
        got = geotiff.read(tif)
        assert np.array_equal(got.data[0], r.data[0, w["row_off"]:w["row_off"] + w["height"],
                                                    w["col_off"]:w["col_off"] + w["width"]])
    for crop in (False, True):
        bb = [-105.45, 40.1, -105.1, 40.45]
        arr, win, tr = streaming.extract_bbox_mosaic(out, bb, ctx=gpu_ctx, crop=crop)
        assert np.array_equal(arr[0], r.data[0, win["row_off"]:win["row_off"] + win["height"],
                                              win["col_off"]:win["col_off"] + win["width"]])
        assert list(tr) == list(geotiff.window_transform(r.transform, win["col_off"], win["row_off"]))
        if crop:  # exactly the bbox's pixel window (clipped to the raster)
            assert win == streaming.bbox_pixel_window(r.transform, bb, r.width, r.height)


def test_raw_frames_sample_dem_matches_fixture(gpu_ctx, golden, tmp_path):
    fx = (golden / "sample_dem.flac").read_bytes()
    m = container.parse_metadata(fx)
    mtime = struct.unpack("<I", base64.b64decode(m.tag("GEOSPATIAL_SPATIAL_INDEX"))[4:8])[0]
    out = tmp_path / "dem_spatial.flac"
    SpatialFLACEncoder(256, gpu_ctx).encode_spatial_flac(golden / "sample_dem.tif", out, date=m.tag("DATE"),
                                                         gzip_mtime=mtime)
    got = out.read_bytes().replace(b"GEOSPATIAL_DATA_MAX=1492.0", b"GEOSPATIAL_DATA_MAX=1493.0")
    assert got == fx


def test_raw_frames_rgb_matches_oracle(gpu_ctx, golden, tmp_path):
    """3-channel 32-bit streams with a few +-1 samples (min/max pixels) -> LPC/FIXED on spikes."""
    out = tmp_path / "rgb_spatial.flac"
    SpatialFLACEncoder(128, gpu_ctx).encode_spatial_flac(golden / "sample_rgb.tif", out, date="2026-01-01",
                                                         gzip_mtime=0)
    r = geotiff.read(golden / "sample_rgb.tif")
    assert out.read_bytes() == P.raw_frames(r.data, list(r.transform), r.crs_string, 128, "2026-01-01", 0)
