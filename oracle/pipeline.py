"""oracle.pipeline -- TEST INFRASTRUCTURE ONLY: whole-file restatement of the reference's outputs.

Builds the exact bytes the reference writes, from the CPU oracle's frames plus an independent restatement
of the container logic it goes through:
  plain convert        converter.py:112-232 (+ mutagen FLAC.save, or the JSON sidecar without mutagen)
  create-streaming     cli.py:620-804 (temp GeoTIFF per tile -> tiff_to_flac -> [u32][JSON][tiles])
  convert --spatial    spatial_encoder.py:136-353 (raw frames, first header rewritten, stale offsets)
mutagen 1.47.0 behaviour restated: VComment.write(framing=False), _writeblocks with one trailing PADDING,
PaddingInfo default = 1024 + content//1000 when the new blocks do not fit the old ones.
Only tests import this module.
"""
from __future__ import annotations

import base64
import gzip
import json
import struct

import numpy as np

from . import oracle as O

VENDOR = "reference libFLAC 1.4.3 20230623"


def _vc(tags):
    v = VENDOR.encode()
    b = struct.pack("<I", len(v)) + v + struct.pack("<I", len(tags))
    for k, val in tags:
        e = (k + "=" + val).encode("utf-8")
        b += struct.pack("<I", len(e)) + e
    return b


def mutagen_save(bare_stream: bytes, tags, tail_after=b"") -> bytes:
    """FLAC(path).clear(); tags...; save() on a file = bare_stream + tail_after (libFLAC metadata: 86 B)."""
    assert bare_stream[:4] == b"fLaC"
    si_len = int.from_bytes(bare_stream[5:8], "big")
    si = bare_stream[8:8 + si_len]
    p = 8 + si_len
    vc_len = int.from_bytes(bare_stream[p + 1:p + 4], "big")
    audio_off = p + 4 + vc_len
    available = audio_off - 4
    vc = _vc(tags)
    blocks = bytes([0]) + len(si).to_bytes(3, "big") + si + bytes([4]) + len(vc).to_bytes(3, "big") + vc
    content = len(bare_stream) - audio_off + len(tail_after)
    padding = available - (len(blocks) + 4)
    high, low = 1024 * 10 + content // 100, 1024 + content // 1000
    pad = (low if padding > high else padding) if padding >= 0 else low
    return b"fLaC" + blocks + bytes([0x81]) + pad.to_bytes(3, "big") + bytes(pad) + bare_stream[audio_off:]


def tags_converter(md):
    return [("TITLE", "Geospatial Raster Data"),
            ("DESCRIPTION", "TIFF raster converted to FLAC with geospatial metadata"),
            ("ENCODER", "FLAC-Raster v0.1.0"),
            ("GEOSPATIAL_CRS", str(md.get("crs", ""))), ("GEOSPATIAL_WIDTH", str(md.get("width", 0))),
            ("GEOSPATIAL_HEIGHT", str(md.get("height", 0))), ("GEOSPATIAL_COUNT", str(md.get("count", 1))),
            ("GEOSPATIAL_DTYPE", str(md.get("dtype", ""))), ("GEOSPATIAL_NODATA", str(md.get("nodata", ""))),
            ("GEOSPATIAL_DATA_MIN", str(md.get("data_min", ""))), ("GEOSPATIAL_DATA_MAX", str(md.get("data_max", ""))),
            ("GEOSPATIAL_TRANSFORM", json.dumps(md.get("transform", []))),
            ("GEOSPATIAL_BOUNDS", json.dumps(md.get("bounds", []))),
            ("GEOSPATIAL_SPATIAL_TILING", str(md.get("spatial_tiling", False)))]


def _affine_mul(t, x, y):
    a, b, c, d, e, f = t[:6]
    return (x * a + y * b + c, x * d + y * e + f)


def _window_transform(t, col, row):
    """rasterio.windows.transform: Affine.translation(x - c, y - f) * t (affine 2.4 composition order)."""
    x, y = _affine_mul(t, col or 0.0, row or 0.0)
    tx, ty = x - t[2], y - t[5]
    a, b, c, d, e, f = t[:6]
    return (1.0 * a + 0.0 * d, 1.0 * b + 0.0 * e, 1.0 * c + 0.0 * f + tx,
            0.0 * a + 1.0 * d, 0.0 * b + 1.0 * e, 0.0 * c + 1.0 * f + ty)


def plain_convert(data: np.ndarray, transform, crs, nodata=None, embed=True, level=5):
    """converter.tiff_to_flac (compression_level=level) -> (flac bytes, sidecar json text or None)."""
    B, H, W = data.shape
    dt = data.dtype
    flat = data.transpose(1, 2, 0).reshape(-1, B)
    pcm, mn, mx, bps = O.normalize(flat)
    sr = O.sample_rate_for(B, H)
    bare = O.stream_header(B, bps, sr) + O.encode_frames(pcm, bps, sr, level=level)
    a, b, c, d, e, f = transform[:6]
    bounds = {"left": c, "bottom": f + e * H, "right": c + a * W, "top": f}
    md = {"width": W, "height": H, "count": B, "dtype": str(dt), "crs": crs, "transform": list(transform),
          "bounds": bounds, "data_min": mn, "data_max": mx, "nodata": nodata, "driver": "GTiff"}
    if embed:
        return mutagen_save(bare, tags_converter(md)), None
    return bare, json.dumps(md, indent=2)


def create_streaming(band: np.ndarray, transform, crs, tile: int) -> bytes:
    """cli.py:668-780 for a single-band (or band-1) raster."""
    H, W = band.shape
    index = {"crs": str(crs), "transform": list(transform), "width": W, "height": H, "tile_size": tile, "frames": []}
    chunks = []
    total = 0
    fid = 0
    for row in range(0, H, tile):
        for col in range(0, W, tile):
            w, h = min(tile, W - col), min(tile, H - row)
            tt = _window_transform(transform, col, row)
            xmin, ymax = tt[2], tt[5]
            xmax, ymin = xmin + (w * tt[0]), ymax + (h * tt[4])
            sub = band[row:row + h, col:col + w]
            flac, _ = plain_convert(sub[None], list(tt) + [0.0, 0.0, 1.0], crs, None, True)
            index["frames"].append({"frame_id": fid, "bbox": [xmin, ymin, xmax, ymax],
                                    "window": {"col_off": col, "row_off": row, "width": w, "height": h},
                                    "byte_offset": total, "byte_size": len(flac)})
            chunks.append(flac)
            total += len(flac)
            fid += 1
    js = json.dumps(index, separators=(",", ":")).encode("utf-8")
    return len(js).to_bytes(4, "big") + js + b"".join(chunks)


def raw_frames(data: np.ndarray, transform, crs, tile: int, date: str, mtime: float, level: int = 5) -> bytes:
    """spatial_encoder.SpatialFLACEncoder.encode_spatial_flac (compression_level=level) + _embed_metadata_in_flac."""
    B, H, W = data.shape
    streams, frames = [], []
    pos = 0
    i = 0
    for row in range(0, H, tile):
        for col in range(0, W, tile):
            h, w = min(row + tile, H) - row, min(col + tile, W) - col
            sub = data[:, row:row + h, col:col + w].reshape(B, h * w).T
            pcm = O.normalize_spatial(np.ascontiguousarray(sub))
            s = O.stream_header(B, 32, 44100) + O.encode_frames(pcm, 32, 44100, level=level)
            xmin, ymax = _affine_mul(transform, col, row)
            xmax, ymin = _affine_mul(transform, col + w, row + h)
            frames.append({"frame_id": i, "bbox": [xmin, ymin, xmax, ymax],
                           "window": {"row_off": row, "col_off": col, "height": h, "width": w},
                           "byte_offset": pos, "byte_size": len(s)})
            streams.append(s)
            pos += len(s)
            i += 1
    index = {"crs": str(crs), "transform": list(transform), "frames": frames}
    comp = gzip.compress(json.dumps(index, separators=(",", ":")).encode("utf-8"), mtime=mtime)
    bounds = [frames[0]["bbox"][0], frames[0]["bbox"][1], frames[-1]["bbox"][2], frames[-1]["bbox"][3]]
    tags = [("TITLE", "Geospatial Raster Data"),
            ("DESCRIPTION", f"TIFF raster converted to spatial FLAC with {len(frames)} tiles"),
            ("ENCODER", "FLAC-Raster v0.1.0"), ("DATE", date), ("GEOSPATIAL_CRS", str(crs)),
            ("GEOSPATIAL_WIDTH", str(W)), ("GEOSPATIAL_HEIGHT", str(H)), ("GEOSPATIAL_COUNT", str(B)),
            ("GEOSPATIAL_DTYPE", str(data.dtype)), ("GEOSPATIAL_DATA_MIN", str(float(np.min(data)))),
            ("GEOSPATIAL_DATA_MAX", str(float(np.max(data)))),
            ("GEOSPATIAL_TRANSFORM", json.dumps(list(transform))), ("GEOSPATIAL_BOUNDS", json.dumps(bounds)),
            ("GEOSPATIAL_SPATIAL_TILING", "true"), ("GEOSPATIAL_TILE_SIZE", str(tile)),
            ("GEOSPATIAL_NUM_TILES", str(len(frames))),
            ("GEOSPATIAL_SPATIAL_INDEX", base64.b64encode(comp).decode("ascii"))]
    tail = b"".join(streams[1:])
    return mutagen_save(streams[0], tags, tail) + tail
