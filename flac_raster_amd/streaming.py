"""Streaming FLAC format (create-streaming / extract-streaming) on the MI355X codec.

Reference: cli.py:620-804 (create_streaming) and cli.py:875-1039 (extract_streaming).
File layout: ``[u32 BE index_len][compact JSON index][tile FLAC 0]...[tile FLAC N-1]``; every tile is a
complete FLAC stream of band 1 (cli.py:699) with the mutagen-embedded geospatial tags of its temporary
GeoTIFF (converter.py:315-349).

Differences from the reference are only in *how*: all tiles are encoded in one GPU call (the reference
loops tiles serially through two temporary files each), and extraction decodes any number of tiles in
one batched GPU call.  ``extract_bbox_mosaic`` is an extension: the reference returns
only the first intersecting tile.
"""
from __future__ import annotations

import json
import logging
import math
import os
import struct
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import container, geotiff
from ._native import Context, default_context
from .converter import audio_params, write_tiff_from_meta

log = logging.getLogger("flac_raster.streaming")


# ----------------------------------------------------------------------------- encode
def tile_grid(height: int, width: int, tile: int) -> List[Tuple[int, int, int, int]]:
    """cli.py:691-696: row-major (col_off, row_off, w, h) windows, edge tiles truncated."""
    out = []
    for row in range(0, height, tile):
        for col in range(0, width, tile):
            out.append((col, row, min(tile, width - col), min(tile, height - row)))
    return out


def tile_transform_and_bbox(transform: geotiff.Affine, col: int, row: int, w: int, h: int):
    """cli.py:702-706 with rasterio's window_transform."""
    tt = geotiff.window_transform(transform, col, row)
    xmin = tt.c
    ymax = tt.f
    xmax = xmin + (w * tt.a)
    ymin = ymax + (h * tt.e)
    return tt, [xmin, ymin, xmax, ymax]


def tile_tags(crs: Optional[str], tt: geotiff.Affine, w: int, h: int, dtype, tmin: float, tmax: float):
    """Tags of the per-tile FLAC (tiff_to_flac on the temporary 1-band GeoTIFF, cli.py:719-733)."""
    bounds = geotiff.GeoRaster(np.empty((1, h, w), dtype=np.uint8), tt).bounds
    md = {
        "width": w, "height": h, "count": 1, "dtype": str(np.dtype(dtype)), "crs": crs,
        "transform": list(tt),
        "bounds": {"left": bounds[0], "bottom": bounds[1], "right": bounds[2], "top": bounds[3]},
        "data_min": tmin, "data_max": tmax, "nodata": None, "driver": "GTiff",
    }
    return container.raster_tags(md)


class TileHeaderBuilder:
    """Per-tile FLAC headers of a streaming file, byte-identical to ``container.mutagen_header(..., tile_tags(...))``
    (the mutagen rewrite of each temporary tile FLAC, converter.py:315-349) at a few microseconds per tile: the
    constant tag entries are encoded once and the per-tile numbers (a C4 file has 6241 tiles but only 79 column
    and 79 row origins) are formatted through a cache.  Checked against the direct path in tests."""

    _PREFIX = (("TITLE", "Geospatial Raster Data"),
               ("DESCRIPTION", "TIFF raster converted to FLAC with geospatial metadata"),
               ("ENCODER", "FLAC-Raster v0.1.0"))

    def __init__(self, crs: Optional[str], dtype, stream_bps: int, sample_rate: int = 44100, blocksize: int = 4096):
        self._si = container.block(container.BLOCK_STREAMINFO,
                                   container.streaminfo(blocksize, sample_rate, 1, stream_bps), False)
        self._vendor = struct.pack("<I", len(container.VENDOR)) + container.VENDOR + struct.pack("<I", 14)
        ent = self._entry
        self._pre = b"".join(ent(k, v) for k, v in self._PREFIX) + ent("GEOSPATIAL_CRS", str(crs))
        self._mid = (ent("GEOSPATIAL_COUNT", "1") + ent("GEOSPATIAL_DTYPE", str(np.dtype(dtype))) +
                     ent("GEOSPATIAL_NODATA", "None"))
        self._tail = ent("GEOSPATIAL_SPATIAL_TILING", "False")
        self._num: Dict[Tuple[type, object, bool], str] = {}
        self._ent: Dict[Tuple[str, str], bytes] = {}

    @staticmethod
    def _entry(k: str, v: str) -> bytes:
        c = k.encode("ascii") + b"=" + v.encode("utf-8")
        return struct.pack("<I", len(c)) + c

    def _js(self, x) -> str:
        """json.dumps of a number (float.__repr__ for finite floats), cached; -0.0 and 0.0 kept apart."""
        key = (type(x), x, math.copysign(1.0, x) < 0 if isinstance(x, float) else False)
        v = self._num.get(key)
        if v is None:
            v = self._num[key] = json.dumps(x)
        return v

    def _cached_entry(self, k: str, v: str) -> bytes:
        e = self._ent.get((k, v))
        if e is None:
            e = self._ent[(k, v)] = self._entry(k, v)
        return e

    def header(self, tt: geotiff.Affine, w: int, h: int, tmin: float, tmax: float, frame_bytes: int) -> bytes:
        js = self._js
        left, bottom, right, top = geotiff.bounds_of(tt, w, h)
        tr = "[" + ", ".join(js(v) for v in tt) + "]"
        bd = '{"left": ' + js(left) + ', "bottom": ' + js(bottom) + ', "right": ' + js(right) + ', "top": ' + \
             js(top) + "}"
        ent = self._entry
        body = b"".join((self._vendor, self._pre, self._cached_entry("GEOSPATIAL_WIDTH", str(w)),
                         self._cached_entry("GEOSPATIAL_HEIGHT", str(h)), self._mid,
                         self._cached_entry("GEOSPATIAL_DATA_MIN", str(tmin)),
                         self._cached_entry("GEOSPATIAL_DATA_MAX", str(tmax)),
                         ent("GEOSPATIAL_TRANSFORM", tr), ent("GEOSPATIAL_BOUNDS", bd), self._tail))
        vc = container.block(container.BLOCK_VORBIS_COMMENT, body, False)
        pad = container.mutagen_padding(86 - 4, len(self._si) + len(vc) + 4, frame_bytes)
        return b"".join((b"fLaC", self._si, vc, container.block(container.BLOCK_PADDING, bytes(pad), True)))


@dataclass
class EncodedTiles:
    """Output of one GPU encode of all band-1 tiles."""
    windows: List[Tuple[int, int, int, int]]
    frames: np.ndarray          # arena: all tiles' frames back to back
    tile_off: np.ndarray        # int64[n+1]
    tile_min: np.ndarray
    tile_max: np.ndarray
    stream_bps: int


def encode_band_tiles(band: np.ndarray, tile_size: int, ctx: Optional[Context] = None,
                      pinned: bool = False) -> EncodedTiles:
    """All band-1 tiles in one GPU launch sequence (the reference's tile loop, cli.py:690-763).  pinned=True: the
    frames land in page-locked memory owned by the returned arena array (Context.pinned: the DMA writes at full
    rate, and the buffer lives as long as any view of it)."""
    H, W = band.shape
    if H == 0 or W == 0:  # an empty shard (more ranks than tile rows): no tiles, nothing to launch
        z = np.zeros(0, dtype=np.float64)
        _, bps = audio_params(1, 1, band.dtype)
        return EncodedTiles([], np.zeros(0, dtype=np.uint8), np.zeros(1, dtype=np.int64), z, z,
                            16 if bps == 16 else 32)
    ctx = ctx or default_context()
    _, bps = audio_params(1, min(tile_size, H), band.dtype)
    d = ctx.make_desc(H, W, band.dtype, nbands=1, tile_h=tile_size, tile_w=tile_size, sample_rate=44100,
                      bits_per_sample=bps)
    arena, off, mn, mx, sbps = ctx.encode_tiles_host(np.ascontiguousarray(band), d, pinned=pinned)
    return EncodedTiles(tile_grid(H, W, tile_size), arena, off, mn, mx, sbps)


def streaming_headers(enc: EncodedTiles, transform: geotiff.Affine, crs: Optional[str], width: int, height: int,
                      tile_size: int, dtype, windows=None, frame_id0: int = 0, byte_offset0: int = 0):
    """Per-tile headers and index entries of `enc`'s tiles (cli.py:702-759): (headers, frames entries, bytes)."""
    windows = enc.windows if windows is None else windows
    hb = TileHeaderBuilder(crs, dtype, enc.stream_bps)
    headers: List[bytes] = []
    frames: List[Dict] = []
    total = byte_offset0
    tile_bytes = np.diff(enc.tile_off)
    for i, (col, row, w, h) in enumerate(windows):
        tt = geotiff.window_transform(transform, col, row)
        # sample rate of the tile: _calculate_audio_params on the (1, h, w) array -> shape0*shape1 = h
        if h >= 1000000:
            raise NotImplementedError("tile heights >= 1e6 rows change the sample rate; re-encode needed")
        fb = int(tile_bytes[i])
        hdr = hb.header(tt, w, h, float(enc.tile_min[i]), float(enc.tile_max[i]), fb)
        xmin, ymax = tt.c, tt.f
        frames.append({"frame_id": frame_id0 + i, "bbox": [xmin, ymax + (h * tt.e), xmin + (w * tt.a), ymax],
                       "window": {"col_off": col, "row_off": row, "width": w, "height": h},
                       "byte_offset": total, "byte_size": len(hdr) + fb})
        headers.append(hdr)
        total += len(hdr) + fb
    return headers, frames, total - byte_offset0


def streaming_head(index: Dict) -> bytes:
    """[u32 BE index length][compact JSON index] (cli.py:769-773)."""
    js = container.index_json(index)
    return struct.pack(">I", len(js)) + js


def assemble_streaming(enc: EncodedTiles, transform: geotiff.Affine, crs: Optional[str], width: int, height: int,
                       tile_size: int, dtype) -> Tuple[bytes, List[bytes], Dict]:
    """Index JSON + per-tile FLAC streams (header bytes + frames) -> (head, tile_streams, index)."""
    headers, frames, _ = streaming_headers(enc, transform, crs, width, height, tile_size, dtype)
    index = {"crs": str(crs), "transform": list(transform), "width": width, "height": height,
             "tile_size": tile_size, "frames": frames}
    streams = [hdr + enc.frames[enc.tile_off[i]:enc.tile_off[i + 1]].tobytes() for i, hdr in enumerate(headers)]
    return streaming_head(index), streams, index


def write_tiles(fd: int, offset: int, headers: Sequence[bytes], enc: EncodedTiles, threads: int = 8) -> None:
    """pwritev of (header, frames) pairs straight from the arena (no per-tile copies), tile ranges in parallel
    threads (os.pwritev releases the GIL); the tiles land back to back from file offset `offset`."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(headers)
    if n == 0:
        return
    mv = memoryview(enc.frames)
    sizes = np.array([len(h) for h in headers], dtype=np.int64) + np.diff(enc.tile_off)
    starts = offset + np.concatenate(([0], np.cumsum(sizes)[:-1]))
    off = enc.tile_off

    def run(a: int, b: int):
        i = a
        while i < b:
            j = min(b, i + 512)  # 1024 iovecs per call (IOV_MAX)
            iov = []
            for k in range(i, j):
                iov.append(headers[k])
                iov.append(mv[off[k]:off[k + 1]])
            want = int(starts[j - 1] + sizes[j - 1] - starts[i])
            done = os.pwritev(fd, iov, int(starts[i]))
            if done != want:  # short write: finish byte-wise
                buf = b"".join(bytes(x) for x in iov)
                while done < want:
                    done += os.pwrite(fd, buf[done:], int(starts[i]) + done)
            i = j

    k = max(1, min(threads, n // 64 or 1))
    bounds = [n * t // k for t in range(k + 1)]
    with ThreadPoolExecutor(k) as ex:
        list(ex.map(lambda t: run(bounds[t], bounds[t + 1]), range(k)))


def create_streaming_array(band: np.ndarray, transform: geotiff.Affine, crs: Optional[str], output: Path,
                           tile_size: int = 1024, ctx: Optional[Context] = None,
                           timings: Optional[Dict[str, float]] = None) -> Dict:
    """cli.py:620-804 on an in-memory band-1 array: one GPU encode of every tile, headers and index on the host,
    tiles written from the arena with parallel pwritev.  Returns the index; `timings` gets the stage seconds."""
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    H, W = band.shape
    # large jobs: frames back into page-locked memory (DMA rate, no page faults) and written from there
    enc = encode_band_tiles(band, tile_size, ctx, pinned=band.nbytes >= (64 << 20))
    t1 = time.perf_counter()
    headers, frames, body = streaming_headers(enc, transform, crs, W, H, tile_size, band.dtype)
    index = {"crs": str(crs), "transform": list(transform), "width": W, "height": H, "tile_size": tile_size,
             "frames": frames}
    head = streaming_head(index)
    t2 = time.perf_counter()
    fd = os.open(output, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        os.ftruncate(fd, len(head) + body)
        t2b = time.perf_counter()  # (truncating an existing file frees its pages: part of the write cost)
        os.pwrite(fd, head, 0)
        write_tiles(fd, len(head), headers, enc)
    finally:
        os.close(fd)
    t3 = time.perf_counter()
    tm.update(encode_s=t1 - t0, index_s=t2 - t1, write_s=t3 - t2, open_truncate_s=t2b - t2, total_s=t3 - t0)
    return index


def create_streaming(input_file: Path, output_file: Path, tile_size: int = 1024,
                     ctx: Optional[Context] = None, timings: Optional[Dict[str, float]] = None,
                     materialize: bool = False) -> Dict:
    """cli.py:620-804 without the console output: writes the streaming file, returns the index.  Band 1 only
    (cli.py:698-699): an uncompressed band-sequential (or single-band) file is encoded straight from its memory map
    (no host copy of the band); otherwise its strips / tiles are decoded.  `timings` gets read_s + the stages of
    create_streaming_array.  materialize=True reads the band into host memory first (read_s is then the whole read;
    otherwise the band's pages are read while the encode copies them, inside encode_s)."""
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    with geotiff.TiffFile(input_file) as tf:
        transform, epsg, _, _ = tf.georef()
        crs = f"EPSG:{epsg}" if epsg else None
        band = None if materialize else tf.band_view(0)
        if band is None:
            band = tf.read_rows(bands=[0])[0]
        tm["read_s"] = time.perf_counter() - t0
        transform = transform or geotiff.Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0)
        index = create_streaming_array(band, transform, crs, output_file, tile_size, ctx, tm)
        del band
    tm["total_s"] = time.perf_counter() - t0
    return index


# ----------------------------------------------------------------------------- read / select
class Source:
    """Local file or HTTP(S) URL with byte-range reads (cli.py:898-919, 1001-1011)."""

    def __init__(self, path_or_url: Union[str, Path]):
        self.src = str(path_or_url)
        self.is_url = self.src.startswith(("http://", "https://"))

    def read(self, start: int, length: int) -> bytes:
        if length <= 0:
            return b""
        if self.is_url:
            import requests
            r = requests.get(self.src, headers={"Range": f"bytes={start}-{start + length - 1}"})
            if r.status_code != 206:
                raise ValueError(f"Server doesn't support range requests: {r.status_code}")
            return r.content
        with open(self.src, "rb") as fh:
            fh.seek(start)
            return fh.read(length)

    def read_ranges(self, ranges: Sequence[Tuple[int, int]]) -> List[bytes]:
        if not self.is_url:
            out = []
            with open(self.src, "rb") as fh:
                for s, n in ranges:
                    fh.seek(s)
                    out.append(fh.read(n))
            return out
        return [self.read(s, n) for s, n in ranges]


def read_index(src: Union[str, Path, Source]) -> Tuple[int, Dict]:
    """Index size and JSON index (cli.py:898-919)."""
    s = src if isinstance(src, Source) else Source(src)
    n = struct.unpack(">I", s.read(0, 4))[0]
    return n, json.loads(s.read(4, n).decode("utf-8"))


def select_frame(index: Dict, tile_id: Optional[int] = None, last: bool = False, center: bool = False,
                 bbox: Optional[Sequence[float]] = None) -> Dict:
    """cli.py:926-990: precedence tile_id > last > center > bbox; bbox = first strict intersection."""
    frames = index["frames"]
    if tile_id is not None:
        for f in frames:
            if f["frame_id"] == tile_id:
                return f
        raise KeyError(f"Tile ID {tile_id} not found")
    if last:
        return max(frames, key=lambda f: f["frame_id"])
    if center:
        bbs = [f["bbox"] for f in frames]
        cx = (min(b[0] for b in bbs) + max(b[2] for b in bbs)) / 2
        cy = (min(b[1] for b in bbs) + max(b[3] for b in bbs)) / 2
        best, dmin = None, float("inf")
        for f in frames:
            fx = (f["bbox"][0] + f["bbox"][2]) / 2
            fy = (f["bbox"][1] + f["bbox"][3]) / 2
            d = ((fx - cx) ** 2 + (fy - cy) ** 2) ** 0.5
            if d < dmin:
                dmin, best = d, f
        return best
    if bbox is not None:
        hit = first_intersecting(index, bbox)
        if hit is None:
            raise LookupError(f"No tiles intersect with bbox {bbox}")
        return hit
    raise ValueError("Must specify --tile-id, --bbox, --center, or --last")


_GRID_CACHE: List[Tuple[tuple, Optional[tuple]]] = []  # (fingerprint, grid) of recently queried indexes


def _grid_key(index: Dict) -> tuple:
    """What the derived grid depends on, besides the frames' bboxes (read live at query time): the index object,
    its frame count and the tile geometry.  No reference to the index is kept (a dropped index is not pinned in
    memory); an index whose geometry or frame list length changes in place gets a new grid."""
    t = index.get("transform")
    return (id(index), id(index["frames"]), len(index["frames"]), index.get("tile_size"), index.get("width"),
            index.get("height"), tuple(t) if t else None)


def _grid_of(index: Dict) -> Optional[tuple]:
    """The row-major tile grid of an index as create-streaming writes it (tile size, columns, rows, the transform's
    scale/offset terms), or None when the index is not that grid.  Derived once per index geometry (a bbox query
    is latency-bound: the per-query dict walks cost more than the tests themselves).  The frames' bboxes are not
    cached: first_intersecting reads them from the index on every query."""
    frames = index["frames"]
    key = _grid_key(index)
    for k, g in _GRID_CACHE:
        if k == key:
            return g
    T, W, H, t = index.get("tile_size"), index.get("width"), index.get("height"), index.get("transform")
    g = None
    if T and W and H and t and len(t) >= 6 and t[1] == 0 and t[3] == 0 and t[0] != 0 and t[4] != 0:
        tc, tr = -(-int(W) // int(T)), -(-int(H) // int(T))
        if len(frames) == tc * tr and all(fr["frame_id"] == k for k, fr in enumerate(frames)):
            g = (int(T), tc, tr, float(t[0]), float(t[2]), float(t[4]), float(t[5]))
    _GRID_CACHE.insert(0, (key, g))
    del _GRID_CACHE[8:]
    return g


def first_intersecting(index: Dict, bbox: Sequence[float]) -> Optional[Dict]:
    """intersecting(index, bbox)[0] (cli.py:976-987) without the linear scan when the index is the
    row-major tile grid create-streaming writes: only tiles within one tile of the bbox's pixel footprint
    are tested, in index order, with the same strict inequalities on the stored bboxes."""
    g = _grid_of(index)
    if g is None:
        hits = intersecting(index, bbox)
        return hits[0] if hits else None
    T, tc, tr, a, c, e, f = g
    frames = index["frames"]
    x0, y0, x1, y1 = bbox
    ca, cb = (x0 - c) / a, (x1 - c) / a
    if cb < ca:
        ca, cb = cb, ca
    ra, rb = (y0 - f) / e, (y1 - f) / e
    if rb < ra:
        ra, rb = rb, ra
    floor = math.floor
    ct0, ct1 = max(0, floor(ca / T) - 1), min(tc - 1, floor(cb / T) + 1)
    rt0, rt1 = max(0, floor(ra / T) - 1), min(tr - 1, floor(rb / T) + 1)
    for r in range(rt0, rt1 + 1):
        k = r * tc
        for cc in range(ct0, ct1 + 1):
            fr = frames[k + cc]
            b = fr["bbox"]
            if x0 < b[2] and x1 > b[0] and y0 < b[3] and y1 > b[1]:
                return fr
    return None


def intersecting(index: Dict, bbox: Sequence[float]) -> List[Dict]:
    """cli.py:976-979 strict-inequality intersection, index order."""
    x0, y0, x1, y1 = bbox
    return [f for f in index["frames"]
            if x0 < f["bbox"][2] and x1 > f["bbox"][0] and y0 < f["bbox"][3] and y1 > f["bbox"][1]]


# ----------------------------------------------------------------------------- decode
class TileDecoder:
    """Batched GPU decode of streaming tiles: one frs_decode_frames call for any number of tiles."""

    def __init__(self, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()

    def decode_streams(self, streams: Sequence[bytes]) -> List[Tuple[np.ndarray, Dict]]:
        metas = [container.parse_metadata(s) for s in streams]
        mds = [container.read_raster_tags(m) for m in metas]
        for m, md in zip(metas, mds):
            if md is None:
                raise ValueError("No metadata found in FLAC file or sidecar file")
            if m.bps not in (16, 32):
                raise ValueError("Only int16/int32 data type is supported")
        out: List[Tuple[np.ndarray, Dict]] = [None] * len(streams)
        # group by (channels, bps, blocksize) so each group is one GPU call
        groups: Dict[Tuple[int, int, int], List[int]] = {}
        for i, m in enumerate(metas):
            groups.setdefault((m.channels, m.bps, m.blocksize), []).append(i)
        for (ch, bps, bs), idx in groups.items():
            blobs = [np.frombuffer(streams[i], dtype=np.uint8)[metas[i].audio_offset:] for i in idx]
            counts = [int(mds[i]["width"]) * int(mds[i]["height"]) for i in idx]
            # one fused decode + de-normalise per raster dtype (tiles of one file share it)
            by_dt: Dict[str, List[int]] = {}
            for j, i in enumerate(idx):
                by_dt.setdefault(str(mds[i]["dtype"]), []).append(j)
            vals_of: Dict[int, np.ndarray] = {}
            for dts, js in by_dt.items():
                sel = [idx[j] for j in js]
                sb = [blobs[j] for j in js]
                so = np.zeros(len(sb) + 1, dtype=np.int64)
                so[1:] = np.cumsum([len(b) for b in sb])
                cnt = [counts[j] for j in js]
                blob = sb[0] if len(sb) == 1 else np.concatenate(sb)  # one tile (extract): no host copy
                allv = self.ctx.decode_tiles_host(blob, so, cnt, channels=ch, bps=bps,
                                                  data_min=[mds[i]["data_min"] for i in sel],
                                                  data_max=[mds[i]["data_max"] for i in sel], dtype=np.dtype(dts),
                                                  blocksize=bs)
                p0 = 0
                for j, n in zip(js, cnt):
                    vals_of[j] = allv[p0:p0 + n]
                    p0 += n
            for j, i in enumerate(idx):
                md = mds[i]
                vals = vals_of[j]
                H, W, C = int(md["height"]), int(md["width"]), int(md["count"])
                arr = vals.reshape(H, W, C).transpose(2, 0, 1) if C > 1 else vals.reshape(1, H, W)
                out[i] = (np.ascontiguousarray(arr), md)
        return out


def fetch_tiles(src: Union[str, Path, Source], frames: Sequence[Dict], index_size: int) -> List[bytes]:
    s = src if isinstance(src, Source) else Source(src)
    return s.read_ranges([(4 + index_size + f["byte_offset"], f["byte_size"]) for f in frames])


def extract_streaming(flac_url: Union[str, Path], output: Path, bbox: Optional[Sequence[float]] = None,
                      tile_id: Optional[int] = None, center: bool = False, last: bool = False,
                      ctx: Optional[Context] = None) -> Dict:
    """cli.py:875-1039: pick one tile, range-read it, decode it and write it as a GeoTIFF."""
    src = Source(flac_url)
    n, index = read_index(src)
    f = select_frame(index, tile_id=tile_id, last=last, center=center, bbox=bbox)
    data = fetch_tiles(src, [f], n)[0]
    (arr, md), = TileDecoder(ctx).decode_streams([data])
    write_tiff_from_meta(Path(output), arr, md)
    return f


def bbox_pixel_window(transform: geotiff.Affine, bbox: Sequence[float], width: int, height: int) -> Dict:
    """Smallest whole-pixel window of a north-up raster that covers bbox [xmin, ymin, xmax, ymax], clipped to the
    raster: columns floor((xmin - c) / a) .. ceil((xmax - c) / a), rows floor((ymax - f) / e) .. ceil((ymin - f) / e).
    Pixel coordinates within 1e-6 of an integer are snapped to it first, so a bbox edge on a pixel (or tile) edge
    does not pull in a sliver pixel through float error (-105.1 -> column 400.0000000000057 for a 0.001 grid)."""
    import math

    def snap(v: float) -> float:
        return float(round(v)) if abs(v - round(v)) < 1e-6 else v
    t = transform
    c0 = math.floor(snap((bbox[0] - t.c) / t.a))
    c1 = math.ceil(snap((bbox[2] - t.c) / t.a))
    r0 = math.floor(snap((bbox[3] - t.f) / t.e))
    r1 = math.ceil(snap((bbox[1] - t.f) / t.e))
    c0, r0 = max(0, c0), max(0, r0)
    c1, r1 = min(width, max(c1, c0)), min(height, max(r1, r0))
    return {"col_off": c0, "row_off": r0, "width": c1 - c0, "height": r1 - r0}


def extract_bbox_mosaic(flac_url: Union[str, Path], bbox: Sequence[float], ctx: Optional[Context] = None,
                        crop: bool = True):
    """Extension: decode every tile intersecting bbox in one GPU batch and mosaic them into
    the raster window they cover, cropped (crop=True) to the whole-pixel window of the bbox itself
    (bbox_pixel_window).  Returns (array (1, h, w), window dict, transform list)."""
    src = Source(flac_url)
    n, index = read_index(src)
    hits = intersecting(index, bbox)
    if not hits:
        raise LookupError(f"No tiles intersect with bbox {bbox}")
    datas = fetch_tiles(src, hits, n)
    dec = TileDecoder(ctx).decode_streams(datas)
    c0 = min(f["window"]["col_off"] for f in hits)
    r0 = min(f["window"]["row_off"] for f in hits)
    c1 = max(f["window"]["col_off"] + f["window"]["width"] for f in hits)
    r1 = max(f["window"]["row_off"] + f["window"]["height"] for f in hits)
    dtype = dec[0][0].dtype
    out = np.zeros((1, r1 - r0, c1 - c0), dtype=dtype)
    for f, (arr, _) in zip(hits, dec):
        w = f["window"]
        out[0, w["row_off"] - r0:w["row_off"] - r0 + w["height"], w["col_off"] - c0:w["col_off"] - c0 + w["width"]] = arr[0]
    t = geotiff.Affine(*index["transform"][:6])
    win = {"col_off": c0, "row_off": r0, "width": c1 - c0, "height": r1 - r0}
    if crop and t.b == 0 and t.d == 0:
        cw = bbox_pixel_window(t, bbox, int(index["width"]), int(index["height"]))
        # (the tiles intersecting the bbox cover its pixel window)
        a0, b0 = max(cw["col_off"], c0), max(cw["row_off"], r0)
        a1 = min(cw["col_off"] + cw["width"], c1)
        b1 = min(cw["row_off"] + cw["height"], r1)
        out = np.ascontiguousarray(out[:, b0 - r0:max(b1, b0) - r0, a0 - c0:max(a1, a0) - c0])
        win = {"col_off": a0, "row_off": b0, "width": max(a1 - a0, 0), "height": max(b1 - b0, 0)}
    wt = geotiff.window_transform(t, win["col_off"], win["row_off"])
    return out, win, list(wt)
