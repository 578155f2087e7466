"""Pin the CPU oracle against the reference's own fixtures (tests/golden = reference test_data/)."""
import base64
import gzip
import json
import struct

import numpy as np
import pytest

from flac_raster_amd import container, geotiff
from oracle import oracle as O
from oracle import pipeline as P


def test_sample_rgb_flac_byte_exact(golden):
    """converter.py plain convert, mutagen absent: 3 channels x 16 frames of libFLAC 1.4.3 level 5."""
    r = geotiff.read(golden / "sample_rgb.tif")
    flac, sidecar = P.plain_convert(r.data, list(r.transform), r.crs_string, r.nodata, embed=False)
    assert flac == (golden / "sample_rgb.flac").read_bytes()
    assert sidecar == (golden / "sample_rgb.json").read_text()


def test_sample_dem_raw_frames_byte_exact_modulo_date(golden):
    """convert --spatial --tile-size 256 (raw frames, 32-bit).  The fixture was made from an older
    sample_dem.tif whose max was 1493 (today 1492); DATE and gzip mtime are taken
    from the fixture."""
    fx = (golden / "sample_dem.flac").read_bytes()
    m = container.parse_metadata(fx)
    comp = base64.b64decode(m.tag("GEOSPATIAL_SPATIAL_INDEX"))
    mtime = struct.unpack("<I", comp[4:8])[0]
    r = geotiff.read(golden / "sample_dem.tif")
    assert r.data.max() == 1492
    mine = P.raw_frames(r.data, list(r.transform), r.crs_string, 256, m.tag("DATE"), mtime)
    assert mine.replace(b"GEOSPATIAL_DATA_MAX=1492.0", b"GEOSPATIAL_DATA_MAX=1493.0") == fx
    # stale offsets: recorded before the first header grew (App. C Q7)
    idx = json.loads(gzip.decompress(comp))
    assert [f["byte_offset"] for f in idx["frames"]] == [0, 8454, 16908, 25362]


def test_all_zero_32bit_block_is_fixed_order0(golden):
    """libFLAC 1.4.3 limit_residual estimator quirk: no CONSTANT subframe for 32-bit zeros."""
    fr = O.encode_frames(np.zeros((4096, 1), np.int32), 32, 44100)
    fx = (golden / "sample_dem.flac").read_bytes()
    assert O.stream_header(1, 32, 44100) + fr == fx[10426:10426 + 86 + len(fr)]


def test_oracle_roundtrip_random_shapes():
    rng = np.random.default_rng(0)
    for n, c in [(4096 * 3 + 100, 1), (5000, 2), (200, 3), (3, 1), (4096, 8)]:
        x = (rng.normal(0, 3000, size=(n, c))).astype(np.int16).astype(np.int32)
        fr = O.encode_frames(x, 16, 44100)
        back = O.decode_frames(fr, c, 16, n + 10)
        assert np.array_equal(back, x)


def test_oracle_wasted_bits_and_constant():
    x = np.zeros((8192, 2), np.int32)
    x[:, 0] = 7
    x[:4096, 1] = np.arange(4096) * 8
    x[4096:, 1] = -32768
    fr = O.encode_frames(x, 16, 44100)
    assert np.array_equal(O.decode_frames(fr, 2, 16, 9000), x)


def test_normalize_matches_numpy():
    """converter.py:56-86 restatement vs numpy itself (numpy 2 NEP 50 semantics are importable here)."""
    rng = np.random.default_rng(3)
    for dt, lo, hi in [(np.uint8, 0, 256), (np.uint16, 0, 65536), (np.int16, -2000, 3000)]:
        a = rng.integers(lo, hi, size=5000).astype(dt)
        pcm, mn, mx, bps = O.normalize(a)
        with np.errstate(over="ignore"):
            ref = ((2.0 * (a - np.min(a)) / (np.max(a) - np.min(a)) - 1.0) * 32767).astype(np.int16)
        assert np.array_equal(pcm, ref.astype(np.int32))
        assert (mn, mx) == (float(a.min()), float(a.max()))


def test_normalize_spatial_matches_numpy():
    rng = np.random.default_rng(4)
    for dt in (np.uint8, np.uint16, np.int16):
        info = np.iinfo(dt)
        a = rng.integers(info.min, info.max, size=3000, endpoint=True).astype(dt)
        a[:2] = [info.min, info.max]
        if dt == np.uint8:
            ref = (a.astype(np.float32) - 127.5) / 127.5
        elif dt == np.uint16:
            ref = (a.astype(np.float32) - 32767.5) / 32767.5
        else:
            ref = a.astype(np.float32) / 32767.0
        assert np.array_equal(O.normalize_spatial(a), ref.astype(np.int32))


def test_denormalize_matches_numpy():
    """converter.py:88-110 on soundfile's pcm/32768 float64 input, numpy fp32 semantics."""
    rng = np.random.default_rng(5)
    pcm = rng.integers(-32768, 32767, size=20000).astype(np.int32)
    for dt, dmin, dmax in [(np.uint8, 1.0, 255.0), (np.int16, 577.0, 1492.0), (np.uint16, 0.0, 65535.0)]:
        audio = pcm.astype(np.float64) / 32768.0
        data_norm = audio.astype(np.float32)
        ref = np.round((data_norm + 1.0) / 2.0 * (dmax - dmin) + dmin).astype(dt)
        assert np.array_equal(O.denormalize_i16(pcm, dmin, dmax, dt), ref)


def test_reconstructed_fixture_roundtrip(golden):
    """sample_rgb.flac -> flac_to_tiff == sample_rgb_reconstructed.tif pixels."""
    flac = (golden / "sample_rgb.flac").read_bytes()
    md = json.loads((golden / "sample_rgb.json").read_text())
    pcm = O.decode_frames(flac[86:], 3, 16, 70000)
    out = O.denormalize_i16(pcm, md["data_min"], md["data_max"], np.uint8)
    rec = geotiff.read(golden / "sample_rgb_reconstructed.tif")
    assert np.array_equal(out.reshape(256, 256, 3).transpose(2, 0, 1), rec.data)
