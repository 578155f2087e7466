"""The drop-in surface: the typer CLI (reference cli.py:32-93, 96-244, 293-406, 620-626, 807-1039) -- options,
defaults, exit code 1 on errors -- and the HTTP Range path (cli.py:898-912, 1001-1006; spatial_encoder.py:384-507)
against a localhost server.  Streaming files for the CPU tests come from the oracle pipeline (test infrastructure);
the GPU tests drive the whole commands."""
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

import numpy as np
import pytest
from typer.testing import CliRunner

from flac_raster_amd import container, geotiff, streaming
from flac_raster_amd.cli import app
from oracle import pipeline as P

runner = CliRunner()


# ------------------------------------------------------------------------------------------------ helpers
def _streaming_file(golden, tmp_path, name="sample_dem", tile=200) -> Path:
    r = geotiff.read(golden / f"{name}.tif")
    out = tmp_path / f"{name}_streaming.flac"
    out.write_bytes(P.create_streaming(r.data[0], list(r.transform), r.crs_string, tile))
    return out


class _Server:
    """Serves one byte string at /f.flac; `ranges=False` ignores Range headers (a server without range support)."""

    def __init__(self, data: bytes, ranges: bool = True):
        self.data, self.ranges, self.requests = data, ranges, []
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_HEAD(self):
                self.send_response(200)
                self.send_header("Content-Length", str(len(outer.data)))
                self.end_headers()

            def do_GET(self):
                rng = self.headers.get("Range")
                outer.requests.append(rng)
                if outer.ranges and rng and rng.startswith("bytes="):
                    a, b = rng[6:].split("-")
                    a, b = int(a), min(int(b), len(outer.data) - 1)
                    body = outer.data[a:b + 1]
                    self.send_response(206)
                    self.send_header("Content-Range", f"bytes {a}-{b}/{len(outer.data)}")
                else:
                    body = outer.data
                    self.send_response(200)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}/f.flac"
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.t.start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


# ------------------------------------------------------------------------------------------------ convert
def test_convert_errors_exit_1(golden, tmp_path):
    assert runner.invoke(app, ["convert", str(tmp_path / "missing.tif")]).exit_code == 1
    bad = tmp_path / "x.png"
    bad.write_bytes(b"x")
    assert runner.invoke(app, ["convert", str(bad)]).exit_code == 1
    out = tmp_path / "o.flac"
    out.write_bytes(b"x")
    r = runner.invoke(app, ["convert", str(golden / "sample_rgb.tif"), "-o", str(out)])
    assert r.exit_code == 1 and "already exists" in r.output
    # -c 0..8 (cli.py:36-37): out-of-range levels are refused by the option's range before any work
    assert runner.invoke(app, ["convert", str(golden / "sample_rgb.tif"), "-c", "9"]).exit_code != 0  # typer range
    assert runner.invoke(app, ["convert", str(golden / "sample_rgb.tif"), "-c", "-1"]).exit_code != 0


# ------------------------------------------------------------------------------------------------ create-streaming
def test_create_streaming_errors_exit_1(golden, tmp_path):
    assert runner.invoke(app, ["create-streaming", str(tmp_path / "missing.tif")]).exit_code == 1
    r = runner.invoke(app, ["create-streaming", str(golden / "sample_dem.flac")])
    assert r.exit_code == 1 and "TIFF" in r.output
    src = tmp_path / "a.tif"
    src.write_bytes((golden / "sample_dem.tif").read_bytes())
    (tmp_path / "a_streaming.flac").write_bytes(b"x")  # the default output name (cli.py:648-650)
    r = runner.invoke(app, ["create-streaming", str(src)])
    assert r.exit_code == 1 and "a_streaming.flac" in r.output


# ------------------------------------------------------------------------------------------------ extract-streaming
def test_extract_streaming_selection_errors_exit_1(golden, tmp_path):
    f = _streaming_file(golden, tmp_path)
    out = tmp_path / "t.tif"
    assert runner.invoke(app, ["extract-streaming", str(f), "-o", str(out), "--bbox", "1,2,3"]).exit_code == 1
    r = runner.invoke(app, ["extract-streaming", str(f), "-o", str(out), "--tile-id", "999"])
    assert r.exit_code == 1 and "999" in r.output
    r = runner.invoke(app, ["extract-streaming", str(f), "-o", str(out), "--bbox", "0,0,1,1"])
    assert r.exit_code == 1 and "No tiles intersect" in r.output
    assert runner.invoke(app, ["extract-streaming", str(f), "-o", str(out)]).exit_code == 1  # no selector


def test_http_range_index_and_tile_reads(golden, tmp_path):
    f = _streaming_file(golden, tmp_path)
    data = f.read_bytes()
    srv = _Server(data)
    try:
        n, index = streaming.read_index(srv.url)
        assert (n, index) == streaming.read_index(f)
        assert srv.requests[:2] == ["bytes=0-3", f"bytes=4-{3 + n}"]  # cli.py:901-912
        fr = index["frames"][3]
        got = streaming.fetch_tiles(srv.url, [fr], n)[0]
        a = 4 + n + fr["byte_offset"]
        assert got == data[a:a + fr["byte_size"]]
        assert srv.requests[-1] == f"bytes={a}-{a + fr['byte_size'] - 1}"  # cli.py:997-1006
    finally:
        srv.close()


def test_http_without_range_support_is_an_error(golden, tmp_path):
    f = _streaming_file(golden, tmp_path)
    srv = _Server(f.read_bytes(), ranges=False)
    try:
        with pytest.raises(ValueError, match="range requests: 200"):
            streaming.read_index(srv.url)
        r = runner.invoke(app, ["extract-streaming", srv.url, "-o", str(tmp_path / "t.tif"), "--tile-id", "0"])
        assert r.exit_code == 1 and "range" in r.output
    finally:
        srv.close()


# ------------------------------------------------------------------------------------------------ raw frames
def test_query_ranges_and_data_on_fixture(golden, tmp_path):
    """query --format ranges/data on sample_dem.flac (the reference's own raw-frames output): index offsets as stored
    (stale by the header growth), merged ranges (spatial_encoder.py:464-484)."""
    fx = golden / "sample_dem.flac"
    from flac_raster_amd.spatial_encoder import SpatialFLACStreamer
    st = SpatialFLACStreamer(fx)
    frames = st.spatial_index.frames
    assert [(f.byte_offset, f.byte_size) for f in frames] == [(0, 8454), (8454, 8454), (16908, 8454), (25362, 8454)]
    b0 = frames[0].bbox
    assert st.get_byte_ranges_for_bbox(b0) == [(0, 8453)]
    everything = (-180.0, -90.0, 180.0, 90.0)
    assert st.get_byte_ranges_for_bbox(everything) == [(0, 33815)]  # four adjacent ranges merged
    assert st.get_byte_ranges_for_bbox((0.0, 0.0, 1.0, 1.0)) == []
    out = tmp_path / "ranges.json"
    r = runner.invoke(app, ["query", str(fx), "--bbox", ",".join(map(str, everything)), "-o", str(out)])
    assert r.exit_code == 0, r.output
    js = json.loads(out.read_text())
    assert js == {"bbox": list(everything), "total_ranges": 1, "total_bytes": 33816,
                  "ranges": [{"start": 0, "end": 33815, "size": 33816}], "http_headers": ["bytes=0-33815"]}
    assert out.read_text() == json.dumps(js, indent=2)
    dat = tmp_path / "data.bin"
    r = runner.invoke(app, ["query", str(fx), "--bbox", ",".join(map(str, b0)), "-f", "data", "-o", str(dat)])
    assert r.exit_code == 0 and dat.read_bytes() == fx.read_bytes()[:8454]
    assert runner.invoke(app, ["query", str(fx), "--bbox", "1,2,3,4", "-f", "xml"]).exit_code == 1
    assert runner.invoke(app, ["query", str(fx), "--bbox", "1,2"]).exit_code == 1
    assert runner.invoke(app, ["query", str(tmp_path / "none.flac"), "--bbox", "1,2,3,4"]).exit_code == 1


def test_streamer_over_http_and_missing_index(golden, tmp_path):
    fx = golden / "sample_dem.flac"
    data = fx.read_bytes()
    srv = _Server(data)
    try:
        from flac_raster_amd.spatial_encoder import SpatialFLACStreamer
        st = SpatialFLACStreamer(srv.url)
        assert srv.requests[0] == "bytes=0-1048575"  # spatial_encoder.py:398
        b = st.spatial_index.frames[2].bbox
        assert st.stream_bbox_data(b) == data[16908:16908 + 8454]
    finally:
        srv.close()
    plain = tmp_path / "plain.flac"  # a FLAC without GEOSPATIAL_SPATIAL_INDEX and no sidecar
    plain.write_bytes((golden / "sample_rgb.flac").read_bytes())
    assert runner.invoke(app, ["spatial-info", str(plain)]).exit_code == 1
    assert runner.invoke(app, ["query", str(plain), "--bbox", "1,2,3,4"]).exit_code == 1


def test_spatial_info_and_info(golden, tmp_path):
    r = runner.invoke(app, ["spatial-info", str(golden / "sample_dem.flac")])
    assert r.exit_code == 0 and "Total frames/tiles: 4" in r.output and "33,816" in r.output
    r = runner.invoke(app, ["info", str(golden / "sample_rgb.tif")])
    assert r.exit_code == 0 and "256 x 256" in r.output and "Bands: 3" in r.output
    r = runner.invoke(app, ["info", str(golden / "sample_dem.flac")])
    assert r.exit_code == 0 and "Embedded Geospatial Metadata" in r.output and "Spatial tiling: Yes" in r.output
    # sidecar fallback (the mutagen-less fixture) and errors
    side = tmp_path / "sample_rgb.flac"
    side.write_bytes((golden / "sample_rgb.flac").read_bytes())
    side.with_suffix(".json").write_text((golden / "sample_rgb.json").read_text())
    r = runner.invoke(app, ["info", str(side)])
    assert r.exit_code == 0 and "from sample_rgb.json" in r.output
    assert runner.invoke(app, ["info", str(tmp_path / "none.flac")]).exit_code == 1
    bad = tmp_path / "x.png"
    bad.write_bytes(b"x")
    assert runner.invoke(app, ["info", str(bad)]).exit_code == 1


# ------------------------------------------------------------------------------------------------ GPU: whole commands
@pytest.mark.gpu
def test_cli_convert_round_trip(golden, tmp_path):
    flac = tmp_path / "rgb.flac"
    assert runner.invoke(app, ["convert", str(golden / "sample_rgb.tif"), "-o", str(flac)]).exit_code == 0
    r = geotiff.read(golden / "sample_rgb.tif")
    assert flac.read_bytes() == P.plain_convert(r.data, list(r.transform), r.crs_string, r.nodata, embed=True)[0]
    tif = tmp_path / "back.tif"
    assert runner.invoke(app, ["convert", str(flac), "-o", str(tif)]).exit_code == 0
    assert np.array_equal(geotiff.read(tif).data, r.data)
    r2 = runner.invoke(app, ["info", str(flac)])
    assert r2.exit_code == 0 and "Audio shape: (65536, 3)" in r2.output


@pytest.mark.gpu
def test_cli_create_and_extract_streaming(golden, tmp_path):
    src = tmp_path / "dem.tif"
    src.write_bytes((golden / "sample_dem.tif").read_bytes())
    r = runner.invoke(app, ["create-streaming", str(src), "--tile-size", "200"])
    assert r.exit_code == 0, r.output
    out = tmp_path / "dem_streaming.flac"  # default name (cli.py:648-650)
    g = geotiff.read(src)
    assert out.read_bytes() == P.create_streaming(g.data[0], list(g.transform), g.crs_string, 200)
    tif = tmp_path / "t.tif"
    r = runner.invoke(app, ["extract-streaming", str(out), "-o", str(tif), "--bbox", "-105.3,40.2,-105.25,40.25"])
    assert r.exit_code == 0, r.output
    n, index = streaming.read_index(out)
    f = streaming.select_frame(index, bbox=[-105.3, 40.2, -105.25, 40.25])
    w = f["window"]
    assert np.array_equal(geotiff.read(tif).data[0], g.data[0, w["row_off"]:w["row_off"] + w["height"],
                                                            w["col_off"]:w["col_off"] + w["width"]])
    srv = _Server(out.read_bytes())  # the same through HTTP Range requests
    try:
        tif2 = tmp_path / "t2.tif"
        r = runner.invoke(app, ["extract-streaming", srv.url, "-o", str(tif2), "--last"])
        assert r.exit_code == 0, r.output
        last = index["frames"][-1]["window"]
        assert np.array_equal(geotiff.read(tif2).data[0], g.data[0, last["row_off"]:, last["col_off"]:])
    finally:
        srv.close()


@pytest.mark.gpu
def test_cli_create_streaming_two_ranks_one_gpu(golden, tmp_path, monkeypatch):
    """--gpus 2 through the local launcher (two processes; on a one-GPU box they share the device and exchange tile
    sizes over the host bootstrap, FRS_COMM_BACKEND=tcp): the file equals the single-process one."""
    monkeypatch.setenv("FRS_COMM_BACKEND", "tcp")
    out = tmp_path / "two.flac"
    r = runner.invoke(app, ["create-streaming", str(golden / "sample_dem.tif"), "-o", str(out), "--tile-size", "128",
                            "--gpus", "2"])
    assert r.exit_code == 0, r.output
    g = geotiff.read(golden / "sample_dem.tif")
    assert out.read_bytes() == P.create_streaming(g.data[0], list(g.transform), g.crs_string, 128)
