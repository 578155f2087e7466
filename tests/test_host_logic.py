"""CPU tests of the product's host-side logic (containers, GeoTIFF, tile selection) -- no GPU calls."""
import json
import os
import struct

import numpy as np
import pytest

from flac_raster_amd import container, geotiff, streaming
from flac_raster_amd.converter import audio_params, raster_metadata
from oracle import pipeline as P


def test_bare_header_matches_fixture(golden):
    assert container.bare_header(3, 16, 44100) == (golden / "sample_rgb.flac").read_bytes()[:86]


def test_mutagen_header_matches_fixture(golden):
    fx = (golden / "sample_dem.flac").read_bytes()
    m = container.parse_metadata(fx)
    content = len(fx) - m.audio_offset
    hdr = container.mutagen_header(1, 32, 44100, m.tags, content)
    assert hdr == fx[:m.audio_offset]


def test_product_container_equals_oracle_restatement(golden):
    r = geotiff.read(golden / "sample_rgb.tif")
    md = raster_metadata(r, 1.0, 255.0)
    tags = container.raster_tags(md)
    assert tags == P.tags_converter(md)
    bare = container.bare_header(3, 16, 44100) + bytes(5000)
    assert container.mutagen_header(3, 16, 44100, tags, 5000) + bytes(5000) == P.mutagen_save(bare, tags)


def test_sidecar_json_matches_fixture(golden):
    r = geotiff.read(golden / "sample_rgb.tif")
    md = raster_metadata(r, 1.0, 255.0)
    assert json.dumps(md, indent=2) == (golden / "sample_rgb.json").read_text()


def test_audio_params_quirk_q3():
    assert audio_params(3, 256, np.uint8) == (44100, 16)
    assert audio_params(4, 300000, np.int16) == (48000, 16)   # bands*height, not pixels
    assert audio_params(1, 512, np.int32) == (44100, 24)


def test_window_transform_and_bbox_match_oracle():
    t = geotiff.Affine(0.0001, 0.0, -120.0, 0.0, -0.0001, 37.0)
    for col, row in [(0, 0), (512, 0), (512, 1024), (37, 91)]:
        tt = geotiff.window_transform(t, col, row)
        assert tt.to_tuple() == P._window_transform(list(t), col, row)


def test_select_frame_semantics():
    idx = {"frames": [
        {"frame_id": 0, "bbox": [0, 10, 10, 20]}, {"frame_id": 1, "bbox": [10, 10, 20, 20]},
        {"frame_id": 2, "bbox": [0, 0, 10, 10]}, {"frame_id": 3, "bbox": [10, 0, 20, 10]}]}
    assert streaming.select_frame(idx, tile_id=2)["frame_id"] == 2
    assert streaming.select_frame(idx, tile_id=2, last=True)["frame_id"] == 2   # tile_id wins
    assert streaming.select_frame(idx, last=True, center=True)["frame_id"] == 3
    assert streaming.select_frame(idx, center=True)["frame_id"] == 0            # first minimum
    assert streaming.select_frame(idx, bbox=[9, 9, 11, 11])["frame_id"] == 0    # first intersecting
    assert streaming.select_frame(idx, bbox=[10, 10, 15, 15])["frame_id"] == 1  # strict: edge-touch excluded
    with pytest.raises(LookupError):
        streaming.select_frame(idx, bbox=[30, 30, 40, 40])
    with pytest.raises(KeyError):
        streaming.select_frame(idx, tile_id=9)


def test_geotiff_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    for dt, count in [(np.uint8, 3), (np.int16, 1), (np.uint16, 4), (np.float32, 2)]:
        a = (rng.random((count, 37, 53)) * 1000).astype(dt)
        t = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
        p = tmp_path / f"x_{np.dtype(dt).name}.tif"
        geotiff.write(p, a, transform=t, epsg=32636, nodata=0)
        r = geotiff.read(p)
        assert np.array_equal(r.data, a) and r.data.dtype == a.dtype
        assert r.transform.to_tuple() == t.to_tuple() and r.epsg == 32636 and r.nodata == 0.0


def test_streaming_header_parse():
    idx = {"crs": "EPSG:4326", "frames": []}
    js = container.index_json(idx)
    n, back = container.parse_streaming_header(struct.pack(">I", len(js)) + js)
    assert n == len(js) and back == idx


def test_first_intersecting_matches_linear_scan():
    """streaming.first_intersecting == intersecting(...)[0] (cli.py:976-987) on a create-streaming grid,
    including bboxes that touch tile edges exactly (strict inequalities)."""
    from flac_raster_amd import geotiff, streaming
    tr = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    H, W, T = 2100, 3000, 512
    frames = []
    for i, (col, row, w, h) in enumerate(streaming.tile_grid(H, W, T)):
        _, bb = streaming.tile_transform_and_bbox(tr, col, row, w, h)
        frames.append({"frame_id": i, "bbox": bb})
    index = {"transform": list(tr) + [0.0, 0.0, 1.0], "width": W, "height": H, "tile_size": T, "frames": frames}
    rng = np.random.default_rng(3)
    left, top = 500000.0, 4000000.0
    right, bottom = left + W * 10, top - H * 10
    edges_x = [left + k * T * 10 for k in range(W // T + 1)]
    edges_y = [top - k * T * 10 for k in range(H // T + 1)]
    for q in range(3000):
        if q % 3 == 0:  # snapped to tile edges
            x0, x1 = sorted(rng.choice(edges_x, 2))
            y0, y1 = sorted(rng.choice(edges_y, 2))
        else:
            x0, x1 = sorted(rng.uniform(left - 5000, right + 5000, 2))
            y0, y1 = sorted(rng.uniform(bottom - 5000, top + 5000, 2))
        bbox = [x0, y0, x1, y1]
        hits = streaming.intersecting(index, bbox)
        got = streaming.first_intersecting(index, bbox)
        assert (got is None and not hits) or (hits and got is hits[0]), bbox
    # an index mutated in place after its first query: a bbox rewritten, then the tile size changed --
    # the grid accelerator follows the live index, never a cached copy of it
    bbox = list(frames[5]["bbox"])
    assert streaming.first_intersecting(index, bbox) is frames[5]
    frames[5]["bbox"] = [b + 1e7 for b in frames[5]["bbox"]]
    hits = streaming.intersecting(index, bbox)
    assert streaming.first_intersecting(index, bbox) is (hits[0] if hits else None) and frames[5] not in hits
    index["tile_size"] = 1024
    assert streaming._grid_of(index) is None  # no longer the 1024-px grid of these 24 frames: linear scan
    assert streaming.first_intersecting(index, bbox) is (hits[0] if hits else None)


@pytest.mark.parametrize("crs,dtype,tr", [
    ("EPSG:32636", np.int16, geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)),
    (None, np.uint8, geotiff.Affine(0.5, 0.1, -0.0, 0.2, -0.5, 0.0)),   # rotated, negative zero
    ("EPSG:4326", np.uint16, geotiff.Affine(1, 0, 0, 0, -1, 10)),       # integer coefficients
])
def test_tile_header_builder_equals_direct_path(crs, dtype, tr):
    """The cached per-tile header builder writes the same bytes as tile_tags + mutagen_header."""
    rng = np.random.default_rng(0)
    grid = streaming.tile_grid(40000, 40000, 512)
    b = streaming.TileHeaderBuilder(crs, dtype, 16)
    for i in rng.integers(0, len(grid), 200):
        col, row, w, h = grid[i]
        tt, _ = streaming.tile_transform_and_bbox(tr, col, row, w, h)
        mn, mx = float(rng.integers(0, 1000)), float(rng.integers(1000, 5000))
        fb = int(rng.integers(0, 10 ** 7))
        ref = container.mutagen_header(1, 16, 44100, streaming.tile_tags(crs, tt, w, h, dtype, mn, mx), fb)
        assert b.header(tt, w, h, mn, mx, fb) == ref


def test_streaming_writer_equals_assembled_bytes(tmp_path):
    """create-streaming's file writer (parallel pwritev from the arena) == head + concatenated tile streams."""
    rng = np.random.default_rng(3)
    H, W, T = 1300, 2100, 256
    grid = streaming.tile_grid(H, W, T)
    sizes = rng.integers(100, 5000, len(grid))
    off = np.concatenate(([0], np.cumsum(sizes))).astype(np.int64)
    enc = streaming.EncodedTiles(grid, rng.integers(0, 256, int(off[-1]), dtype=np.uint8), off,
                                 rng.random(len(grid)) * 100, 100 + rng.random(len(grid)) * 100, 16)
    tr = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    head, streams, index = streaming.assemble_streaming(enc, tr, "EPSG:32636", W, H, T, np.int16)
    headers, frames, body = streaming.streaming_headers(enc, tr, "EPSG:32636", W, H, T, np.int16)
    assert frames == index["frames"] and body == sum(len(s) for s in streams)
    out = tmp_path / "s.flac"
    fd = os.open(out, os.O_WRONLY | os.O_CREAT)
    streaming.write_tiles(fd, len(head), headers, enc, threads=4)
    os.pwrite(fd, head, 0)
    os.close(fd)
    assert out.read_bytes() == head + b"".join(streams)


def test_tiff_windowed_rows_equal_full_read(tmp_path, golden):
    """TiffFile.read_rows decodes only the chunks under the rows and equals the slice of the full read, for
    strips / tiles, chunky / planar, uncompressed / deflate (+ horizontal predictor), and the fixtures."""
    import numpy as np
    from flac_raster_amd import geotiff
    rng = np.random.default_rng(5)
    data = rng.integers(-3000, 3000, size=(3, 77, 91)).astype(np.int16)
    paths = [golden / f"{n}.tif" for n in ("sample_rgb", "sample_dem", "sample_multispectral")]
    for i, kw in enumerate([{}, dict(compress="deflate"), dict(compress="deflate", predictor=2),
                            dict(tile=32), dict(tile=16, compress="deflate", predictor=2), dict(planar=2),
                            dict(planar=2, tile=32, compress="deflate")]):
        p = tmp_path / f"w{i}.tif"
        geotiff.write(p, data, geotiff.Affine(2.0, 0.0, 10.0, 0.0, -2.0, 50.0), 32636, **kw)
        assert np.array_equal(geotiff.read(p).data, data), kw
        paths.append(p)
    for p in paths:
        full = geotiff.read(p)
        with geotiff.TiffFile(p) as tf:
            H = tf.height
            for r0, r1 in ((0, 1), (5, 40), (H - 3, H), (0, H), (17, 18)):
                for bands in (None, [0], [tf.count - 1]):
                    got = tf.read_rows(r0, r1, bands)
                    sel = full.data if bands is None else full.data[bands]
                    assert np.array_equal(got, sel[:, r0:r1]), (p.name, r0, r1, bands)
            assert tf.georef()[0] == full.transform


def test_bbox_pixel_window_covers_bbox():
    """Mosaic crop (extension): the smallest whole-pixel window covering the bbox, clipped."""
    from flac_raster_amd import geotiff, streaming
    t = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    assert streaming.bbox_pixel_window(t, [500015, 3999900, 500101, 3999985], 100, 100) == \
        {"col_off": 1, "row_off": 1, "width": 10, "height": 9}
    assert streaming.bbox_pixel_window(t, [500000, 3999900, 500100, 4000000], 100, 100) == \
        {"col_off": 0, "row_off": 0, "width": 10, "height": 10}
    # clipped at the raster edge
    assert streaming.bbox_pixel_window(t, [499000, 3990000, 500050, 4001000], 100, 100) == \
        {"col_off": 0, "row_off": 0, "width": 5, "height": 100}
    # bbox edges on pixel edges through float error (sample_dem.tif's 0.001-degree grid): no sliver pixel
    d = geotiff.Affine(0.001, 0.0, -105.5, 0.0, -0.001, 40.5)
    assert streaming.bbox_pixel_window(d, [-105.45, 40.1, -105.1, 40.45], 512, 512) == \
        {"col_off": 50, "row_off": 50, "width": 350, "height": 350}
