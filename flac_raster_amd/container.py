"""FLAC container bytes around the GPU-coded frames (host side; text/metadata, not sample arithmetic).

Restates, byte for byte:
  * libFLAC 1.4.3's stream header as written through pyflac's StreamEncoder: "fLaC", STREAMINFO with
    min/max framesize 0, total samples 0 and MD5 0 (no seek callback), and a last VORBIS_COMMENT with
    the vendor string only -- pinned by tests/golden/sample_rgb.flac bytes 0..85;
  * mutagen 1.47.0 ``FLAC.save()`` after ``clear()`` + tag assignment (reference converter.py:315-349,
    spatial_encoder.py:296-353): STREAMINFO, VORBIS_COMMENT (vendor kept, tags in assignment order),
    then one PADDING block whose size follows mutagen's PaddingInfo default rule -- pinned by
    tests/golden/sample_dem.flac (951-byte VORBIS_COMMENT + 1057-byte PADDING);
  * the streaming container ``[u32 BE len][compact JSON index][tile streams]`` (cli.py:679-686, 748-780).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

VENDOR = b"reference libFLAC 1.4.3 20230623"  # libFLAC 1.4.3 vendor string (sonos-pyflac.txt:150)

BLOCK_STREAMINFO = 0
BLOCK_PADDING = 1
BLOCK_VORBIS_COMMENT = 4


def streaminfo(blocksize: int, sample_rate: int, channels: int, bps: int, min_framesize: int = 0,
               max_framesize: int = 0, total_samples: int = 0, md5: bytes = bytes(16)) -> bytes:
    """34-byte STREAMINFO payload (RFC 9639 8.2)."""
    v = (sample_rate << 44) | ((channels - 1) << 41) | ((bps - 1) << 36) | (total_samples & ((1 << 36) - 1))
    return (struct.pack(">HH", blocksize, blocksize) + min_framesize.to_bytes(3, "big") +
            max_framesize.to_bytes(3, "big") + v.to_bytes(8, "big") + md5)


def block(code: int, payload: bytes, last: bool) -> bytes:
    if len(payload) >= 1 << 24:
        raise ValueError("metadata block too large")
    return bytes([code | (0x80 if last else 0)]) + len(payload).to_bytes(3, "big") + payload


def vorbis_comment(tags: Sequence[Tuple[str, str]], vendor: bytes = VENDOR) -> bytes:
    """VORBIS_COMMENT payload as mutagen's VComment.write(framing=False) emits it."""
    out = [struct.pack("<I", len(vendor)), vendor, struct.pack("<I", len(tags))]
    for k, v in tags:
        c = k.encode("ascii") + b"=" + v.encode("utf-8")
        out.append(struct.pack("<I", len(c)))
        out.append(c)
    return b"".join(out)


def bare_header(channels: int, bps: int, sample_rate: int, blocksize: int = 4096) -> bytes:
    """Stream header exactly as libFLAC writes it through pyflac (86 bytes)."""
    return (b"fLaC" + block(BLOCK_STREAMINFO, streaminfo(blocksize, sample_rate, channels, bps), False) +
            block(BLOCK_VORBIS_COMMENT, vorbis_comment([]), True))


def mutagen_padding(available: int, blocks_size: int, content_size: int) -> int:
    """mutagen 1.47 PaddingInfo._get_default_padding (available/blocks_size include the padding header)."""
    padding = available - blocks_size
    high = 1024 * 10 + content_size // 100
    low = 1024 + content_size // 1000
    if padding >= 0:
        return low if padding > high else padding
    return low


def mutagen_header(channels: int, bps: int, sample_rate: int, tags: Sequence[Tuple[str, str]], content_size: int,
                   blocksize: int = 4096, vendor: bytes = VENDOR, original_header_size: int = 86) -> bytes:
    """Header after mutagen's FLAC.save() on a libFLAC stream: STREAMINFO, VORBIS_COMMENT(tags), PADDING.

    ``content_size`` = bytes after the original metadata (mutagen: file size - audio offset), i.e. the
    frames of this stream (plus any further concatenated streams, as in the raw-frames format).
    """
    si = block(BLOCK_STREAMINFO, streaminfo(blocksize, sample_rate, channels, bps), False)
    vc = block(BLOCK_VORBIS_COMMENT, vorbis_comment(tags, vendor), False)
    available = original_header_size - 4  # metadata bytes after "fLaC" in the libFLAC stream
    blocks_size = len(si) + len(vc) + 4
    pad = mutagen_padding(available, blocks_size, content_size)
    return b"fLaC" + si + vc + block(BLOCK_PADDING, bytes(pad), True)


@dataclass
class StreamMeta:
    sample_rate: int
    channels: int
    bps: int
    blocksize: int
    total_samples: int
    vendor: bytes
    tags: List[Tuple[str, str]] = field(default_factory=list)
    audio_offset: int = 0  # first frame byte

    def tag(self, key: str) -> Optional[str]:
        k = key.upper()
        for kk, v in self.tags:
            if kk.upper() == k:
                return v
        return None


def parse_metadata(buf: bytes, offset: int = 0) -> StreamMeta:
    """Parse "fLaC" + metadata blocks starting at buf[offset]."""
    if buf[offset:offset + 4] != b"fLaC":
        raise ValueError("not a FLAC stream (missing fLaC marker)")
    p = offset + 4
    meta = None
    tags: List[Tuple[str, str]] = []
    vendor = b""
    while True:
        if p + 4 > len(buf):
            raise ValueError("truncated FLAC metadata")
        hdr = buf[p]
        last, code = hdr >> 7, hdr & 0x7F
        n = int.from_bytes(buf[p + 1:p + 4], "big")
        payload = buf[p + 4:p + 4 + n]
        if len(payload) < n:
            raise ValueError("truncated FLAC metadata block")
        if code == BLOCK_STREAMINFO:
            v = int.from_bytes(payload[10:18], "big")
            meta = dict(blocksize=struct.unpack(">H", payload[2:4])[0], sample_rate=v >> 44,
                        channels=((v >> 41) & 7) + 1, bps=((v >> 36) & 31) + 1, total_samples=v & ((1 << 36) - 1))
        elif code == BLOCK_VORBIS_COMMENT:
            vl = struct.unpack("<I", payload[:4])[0]
            vendor = payload[4:4 + vl]
            q = 4 + vl
            cnt = struct.unpack("<I", payload[q:q + 4])[0]
            q += 4
            for _ in range(cnt):
                ln = struct.unpack("<I", payload[q:q + 4])[0]
                c = payload[q + 4:q + 4 + ln].decode("utf-8", errors="replace")
                q += 4 + ln
                k, _, val = c.partition("=")
                tags.append((k, val))
        p += 4 + n
        if last:
            break
    if meta is None:
        raise ValueError("FLAC stream without STREAMINFO")
    return StreamMeta(vendor=vendor, tags=tags, audio_offset=p, **meta)


# ----------------------------------------------------------------------------- raster tag blocks
def py_str(v) -> str:
    """str() of a metadata value as the reference's f-string/str() would render it."""
    return str(v)


def raster_tags(metadata: Dict) -> List[Tuple[str, str]]:
    """converter.py:327-346 -- the 14 tags _embed_metadata_in_flac writes, in order."""
    return [
        ("TITLE", "Geospatial Raster Data"),
        ("DESCRIPTION", "TIFF raster converted to FLAC with geospatial metadata"),
        ("ENCODER", "FLAC-Raster v0.1.0"),
        ("GEOSPATIAL_CRS", str(metadata.get("crs", ""))),
        ("GEOSPATIAL_WIDTH", str(metadata.get("width", 0))),
        ("GEOSPATIAL_HEIGHT", str(metadata.get("height", 0))),
        ("GEOSPATIAL_COUNT", str(metadata.get("count", 1))),
        ("GEOSPATIAL_DTYPE", str(metadata.get("dtype", ""))),
        ("GEOSPATIAL_NODATA", str(metadata.get("nodata", ""))),
        ("GEOSPATIAL_DATA_MIN", str(metadata.get("data_min", ""))),
        ("GEOSPATIAL_DATA_MAX", str(metadata.get("data_max", ""))),
        ("GEOSPATIAL_TRANSFORM", json.dumps(metadata.get("transform", []))),
        ("GEOSPATIAL_BOUNDS", json.dumps(metadata.get("bounds", []))),
        ("GEOSPATIAL_SPATIAL_TILING", str(metadata.get("spatial_tiling", False))),
    ]


def read_raster_tags(meta: StreamMeta) -> Optional[Dict]:
    """converter.py:375-414 (_read_embedded_metadata) on already-parsed tags."""
    if meta.tag("GEOSPATIAL_CRS") is None:
        return None
    fields = ["GEOSPATIAL_CRS", "GEOSPATIAL_WIDTH", "GEOSPATIAL_HEIGHT", "GEOSPATIAL_COUNT", "GEOSPATIAL_DTYPE",
              "GEOSPATIAL_NODATA", "GEOSPATIAL_DATA_MIN", "GEOSPATIAL_DATA_MAX", "GEOSPATIAL_TRANSFORM",
              "GEOSPATIAL_BOUNDS", "GEOSPATIAL_SPATIAL_TILING"]
    out: Dict = {}
    for f in fields:
        value = meta.tag(f)
        if value is None:
            continue
        key = f.replace("GEOSPATIAL_", "").lower()
        if key in ("width", "height", "count"):
            out[key] = int(value) if value else 0
        elif key in ("data_min", "data_max"):
            out[key] = float(value) if value else 0.0
        elif key in ("transform", "bounds"):
            out[key] = json.loads(value) if value else []
        elif key == "spatial_tiling":
            out[key] = value.lower() == "true"
        elif key == "nodata":
            out[key] = None if value == "None" else float(value) if value else None
        else:
            out[key] = value
    return out


# ----------------------------------------------------------------------------- streaming container
def index_json(index: Dict) -> bytes:
    """json.dumps(spatial_index, separators=(',', ':')).encode('utf-8') (cli.py:771)."""
    return json.dumps(index, separators=(",", ":")).encode("utf-8")


def parse_streaming_header(head: bytes) -> Tuple[int, Dict]:
    """[4 bytes BE index size][JSON] -> (index_size, index) (cli.py:914-919)."""
    if len(head) < 4:
        raise ValueError("truncated streaming header")
    n = struct.unpack(">I", head[:4])[0]
    if len(head) < 4 + n:
        raise ValueError("truncated streaming index")
    return n, json.loads(head[4:4 + n].decode("utf-8"))
