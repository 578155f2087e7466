"""Raw-frames spatial FLAC (`convert --spatial`) -- reference spatial_encoder.py:21-373 on the MI355X codec.

Format: one complete 32-bit FLAC stream per tile (all bands interleaved), streams
concatenated; the FIRST stream's header is rewritten by mutagen with 17 tags including DATE and the
gzip+base64 spatial index.  Index byte offsets are recorded before that rewrite (stale by the header
growth, App. C Q7) -- reproduced as-is.  Samples are the spatial encoder's float32 normalisation cast
to int32 by pyflac, i.e. {-1, 0, 1} (App. C Q1): the GPU codec computes exactly that (FRS_NORM_SPATIAL).
"""
from __future__ import annotations

import base64
import gzip
import json
import logging
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import container, geotiff
from ._native import Context, default_context
from .converter import check_level

log = logging.getLogger("flac_raster.spatial_encoder")


@dataclass
class Window:
    """rasterio.windows.Window(col_off, row_off, width, height)"""
    col_off: int
    row_off: int
    width: int
    height: int


class SpatialFrame:
    """spatial_encoder.py:21-45"""

    def __init__(self, frame_id: int, bbox: Tuple[float, float, float, float], window: Window,
                 byte_offset: int = 0, byte_size: int = 0):
        self.frame_id = frame_id
        self.bbox = bbox
        self.window = window
        self.byte_offset = byte_offset
        self.byte_size = byte_size

    def to_dict(self) -> Dict:
        return {"frame_id": self.frame_id, "bbox": self.bbox,
                "window": {"row_off": self.window.row_off, "col_off": self.window.col_off,
                           "height": self.window.height, "width": self.window.width},
                "byte_offset": self.byte_offset, "byte_size": self.byte_size}


class SpatialIndex:
    """spatial_encoder.py:48-78"""

    def __init__(self, frames: List[SpatialFrame], crs: Optional[str], transform: geotiff.Affine):
        self.frames = frames
        self.crs = crs
        self.transform = transform
        self.total_bytes = sum(f.byte_size for f in frames)

    def query_bbox(self, bbox) -> List[SpatialFrame]:
        xmin, ymin, xmax, ymax = bbox
        return [f for f in self.frames
                if xmin < f.bbox[2] and xmax > f.bbox[0] and ymin < f.bbox[3] and ymax > f.bbox[1]]

    def to_dict(self) -> Dict:
        return {"crs": str(self.crs), "transform": list(self.transform), "frames": [f.to_dict() for f in self.frames]}


class SpatialFLACEncoder:
    """spatial_encoder.py:81-373"""

    def __init__(self, tile_size: int = 512, ctx: Optional[Context] = None):
        self.tile_size = tile_size
        self.logger = log
        self.frames: List[SpatialFrame] = []
        self._ctx = ctx

    @property
    def ctx(self) -> Context:
        if self._ctx is None:
            self._ctx = default_context()
        return self._ctx

    def _calculate_tiles(self, height: int, width: int) -> List[Tuple[int, int, int, int]]:
        """(row_off, col_off, h, w), row-major (spatial_encoder.py:92-103)."""
        tiles = []
        for r in range(0, height, self.tile_size):
            for c in range(0, width, self.tile_size):
                tiles.append((r, c, min(r + self.tile_size, height) - r, min(c + self.tile_size, width) - c))
        return tiles

    @staticmethod
    def _tile_to_bbox(row_off, col_off, height, width, transform: geotiff.Affine):
        """spatial_encoder.py:105-112"""
        xmin, ymax = transform * (col_off, row_off)
        xmax, ymin = transform * (col_off + width, row_off + height)
        return (xmin, ymin, xmax, ymax)

    def encode_spatial_flac(self, tiff_path: Path, flac_path: Path, compression_level: int = 5,
                            enable_streaming: bool = True, date: Optional[str] = None,
                            gzip_mtime: Optional[float] = None) -> SpatialIndex:
        """spatial_encoder.py:136-227 (+ _embed_metadata_in_flac :296-353).  ``date`` / ``gzip_mtime`` default
        to now, as in the reference (which is therefore not byte-reproducible run to run, App. C Q8)."""
        r = geotiff.read(tiff_path)
        check_level(compression_level, r.count)
        transform = r.transform or geotiff.Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0)
        data = np.ascontiguousarray(r.data)
        B, H, W = data.shape
        tiles = self._calculate_tiles(H, W)
        d = self.ctx.make_desc(H, W, data.dtype, nbands=B, tile_h=self.tile_size, tile_w=self.tile_size,
                               sample_rate=44100, bits_per_sample=24, norm_mode=1, compression_level=compression_level)
        arena, off, mn, mx, sbps = self.ctx.encode_tiles_host(data, d)
        bare = container.bare_header(B, sbps, 44100)
        self.frames = []
        streams = []
        pos = 0
        for i, (ro, co, th, tw) in enumerate(tiles):
            s = bare + arena[off[i]:off[i + 1]].tobytes()
            f = SpatialFrame(i, self._tile_to_bbox(ro, co, th, tw, transform), Window(co, ro, tw, th), pos, len(s))
            self.frames.append(f)
            streams.append(s)
            pos += len(s)
        index = SpatialIndex(self.frames, r.crs_string, transform)
        tags = self._tags(index, r, tiles, float(np.min(mn)), float(np.max(mx)), date, gzip_mtime)
        first = streams[0]
        content = len(first) - len(bare) + sum(len(s) for s in streams[1:])
        hdr = container.mutagen_header(B, sbps, 44100, tags, content)
        with open(flac_path, "wb") as fh:
            fh.write(hdr)
            fh.write(first[len(bare):])
            for s in streams[1:]:
                fh.write(s)
        return index

    def _tags(self, index: SpatialIndex, r: geotiff.GeoRaster, tiles, dmin: float, dmax: float,
              date: Optional[str], gzip_mtime: Optional[float]):
        f0, fl = index.frames[0], index.frames[-1]
        bounds = [f0.bbox[0], f0.bbox[1], fl.bbox[2], fl.bbox[3]]
        spatial_json = json.dumps(index.to_dict(), separators=(",", ":"))
        comp = gzip.compress(spatial_json.encode("utf-8"), mtime=gzip_mtime if gzip_mtime is not None else time.time())
        return [
            ("TITLE", "Geospatial Raster Data"),
            ("DESCRIPTION", f"TIFF raster converted to spatial FLAC with {len(tiles)} tiles"),
            ("ENCODER", "FLAC-Raster v0.1.0"),
            ("DATE", date if date is not None else str(np.datetime64("now", "D"))),
            ("GEOSPATIAL_CRS", str(index.crs)),
            ("GEOSPATIAL_WIDTH", str(r.width)),
            ("GEOSPATIAL_HEIGHT", str(r.height)),
            ("GEOSPATIAL_COUNT", str(r.count)),
            ("GEOSPATIAL_DTYPE", str(r.dtype)),
            ("GEOSPATIAL_DATA_MIN", str(dmin)),
            ("GEOSPATIAL_DATA_MAX", str(dmax)),
            ("GEOSPATIAL_TRANSFORM", json.dumps(list(index.transform))),
            ("GEOSPATIAL_BOUNDS", json.dumps(bounds)),
            ("GEOSPATIAL_SPATIAL_TILING", "true"),
            ("GEOSPATIAL_TILE_SIZE", str(self.tile_size)),
            ("GEOSPATIAL_NUM_TILES", str(len(tiles))),
            ("GEOSPATIAL_SPATIAL_INDEX", base64.b64encode(comp).decode("ascii")),
        ]


def load_spatial_index(flac_path: Path) -> SpatialIndex:
    """Embedded GEOSPATIAL_SPATIAL_INDEX (spatial_encoder.py:384-437, local files)."""
    meta = container.parse_metadata(Path(flac_path).read_bytes()[:1 << 20])
    enc = meta.tag("GEOSPATIAL_SPATIAL_INDEX")
    if enc is None:
        side = Path(flac_path).with_suffix(".spatial.json")
        data = json.loads(side.read_text())
    else:
        data = json.loads(gzip.decompress(base64.b64decode(enc.encode("ascii"))).decode("utf-8"))
    frames = [SpatialFrame(fd["frame_id"], tuple(fd["bbox"]),
                           Window(fd["window"]["col_off"], fd["window"]["row_off"], fd["window"]["width"],
                                  fd["window"]["height"]), fd["byte_offset"], fd["byte_size"])
              for fd in data["frames"]]
    return SpatialIndex(frames, data["crs"], geotiff.Affine(*data["transform"][:6]))


class SpatialFLACStreamer:
    """HTTP-range streaming of raw-frames spatial FLAC files (reference spatial_encoder.py:376-507).

    The index comes from the embedded GEOSPATIAL_SPATIAL_INDEX tag (for URLs: the first MiB through one Range
    request, spatial_encoder.py:398) or the ``.spatial.json`` sidecar.  Its byte offsets are the reference's
    pre-rewrite offsets (stale by the first stream's header growth) and are served as they are.
    One divergence: the reference's ``stream_bbox_data`` calls ``.startswith`` on a ``Path`` and fails for local
    files (Q7); here local paths (str or Path) are read with seek/read.
    """

    def __init__(self, flac_path):
        self.flac_path = flac_path
        self.is_url = isinstance(flac_path, str) and flac_path.startswith(("http://", "https://"))
        self.logger = logging.getLogger("flac_raster.spatial_streamer")
        self.spatial_index = self._load_spatial_index()

    def _load_spatial_index(self) -> SpatialIndex:
        data = None
        try:
            if self.is_url:
                import requests
                r = requests.get(self.flac_path, headers={"Range": "bytes=0-1048575"}, stream=True)
                r.raise_for_status()
                head = r.content
            else:
                with open(self.flac_path, "rb") as fh:
                    head = fh.read(1 << 20)
            enc = container.parse_metadata(head).tag("GEOSPATIAL_SPATIAL_INDEX")
            if enc is None:
                raise ValueError("No embedded spatial index found")
            self.logger.info("Reading spatial index from embedded FLAC metadata")
            data = json.loads(gzip.decompress(base64.b64decode(enc.encode("ascii"))).decode("utf-8"))
        except Exception as e:  # reference: any failure -> sidecar (spatial_encoder.py:428-440)
            self.logger.warning(f"Failed to read embedded metadata: {e}")
            self.logger.info("Falling back to sidecar file")
            side = Path(self.flac_path).with_suffix(".spatial.json")
            if not side.exists():
                raise FileNotFoundError(f"Spatial index not found in FLAC metadata or sidecar file: {side}")
            data = json.loads(side.read_text())
        frames = [SpatialFrame(fd["frame_id"], tuple(fd["bbox"]),
                               Window(fd["window"]["col_off"], fd["window"]["row_off"], fd["window"]["width"],
                                      fd["window"]["height"]), fd["byte_offset"], fd["byte_size"])
                  for fd in data["frames"]]
        return SpatialIndex(frames, data["crs"], geotiff.Affine(*data["transform"][:6]))

    def get_byte_ranges_for_bbox(self, bbox) -> List[Tuple[int, int]]:
        """Inclusive (start, end) byte ranges of the frames intersecting bbox, sorted and merged when overlapping or
        adjacent (spatial_encoder.py:464-484)."""
        ranges = sorted((f.byte_offset, f.byte_offset + f.byte_size - 1)
                        for f in self.spatial_index.query_bbox(bbox) if f.byte_size > 0)
        merged: List[Tuple[int, int]] = []
        for start, end in ranges:
            if merged and start <= merged[-1][1] + 1:
                merged[-1] = (merged[-1][0], max(merged[-1][1], end))
            else:
                merged.append((start, end))
        self.logger.info(f"Found {len(merged)} byte ranges for bbox {bbox}")
        return merged

    def stream_bbox_data(self, bbox) -> bytes:
        """The bytes of those ranges, concatenated (spatial_encoder.py:486-507)."""
        chunks = []
        ranges = self.get_byte_ranges_for_bbox(bbox)
        if self.is_url:
            import requests
            for start, end in ranges:
                r = requests.get(self.flac_path, headers={"Range": f"bytes={start}-{end}"})
                r.raise_for_status()
                chunks.append(r.content)
        else:
            with open(self.flac_path, "rb") as fh:
                for start, end in ranges:
                    fh.seek(start)
                    chunks.append(fh.read(end - start + 1))
        return b"".join(chunks)
