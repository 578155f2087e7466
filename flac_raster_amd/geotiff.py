"""Minimal GeoTIFF reader/writer (rasterio/GDAL are not available in this image).

Covers what the reference's hot path touches through rasterio (converter.py:137-150, 305-309;
cli.py:668-729): band-sequential pixel arrays, dtype, width/height/count, the affine transform
(ModelPixelScale + ModelTiepoint, or ModelTransformation), the EPSG code of the CRS, nodata
(GDAL_NODATA tag) and ``bounds``.  Reading: strips or tiles, chunky or planar, uncompressed, Deflate
(8 / 32946), LZW (5) and PackBits (32773), horizontal predictor 2.  Writing: uncompressed strips in
GDAL's GTiff layout (PlanarConfiguration 1 for multi-band, ~8 KB strips), little-endian, classic TIFF or
BigTIFF when larger than 4 GB.
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

_TYPES = {1: ("B", 1), 2: ("s", 1), 3: ("H", 2), 4: ("I", 4), 5: ("II", 8), 6: ("b", 1), 7: ("B", 1),
          8: ("h", 2), 9: ("i", 4), 10: ("ii", 8), 11: ("f", 4), 12: ("d", 8), 16: ("Q", 8), 17: ("q", 8),
          18: ("Q", 8)}


@dataclass
class Affine:
    """affine.Affine subset (a, b, c, d, e, f) with rasterio's 9-tuple iteration order."""
    a: float
    b: float
    c: float
    d: float
    e: float
    f: float

    def __iter__(self):
        return iter((self.a, self.b, self.c, self.d, self.e, self.f, 0.0, 0.0, 1.0))

    def __mul__(self, other):
        if isinstance(other, Affine):
            # affine 2.4.0 Affine.__mul__ composition, same operation order
            sa, sb, sc, sd, se, sf = self.a, self.b, self.c, self.d, self.e, self.f
            oa, ob, oc, od, oe, of = other.a, other.b, other.c, other.d, other.e, other.f
            return Affine(sa * oa + sb * od, sa * ob + sb * oe, sa * oc + sb * of + sc,
                          sd * oa + se * od, sd * ob + se * oe, sd * oc + se * of + sf)
        vx, vy = other
        return (vx * self.a + vy * self.b + self.c, vx * self.d + vy * self.e + self.f)

    @staticmethod
    def translation(x: float, y: float) -> "Affine":
        return Affine(1.0, 0.0, x, 0.0, 1.0, y)

    def to_tuple(self):
        return (self.a, self.b, self.c, self.d, self.e, self.f)


def window_transform(transform: Affine, col_off: int, row_off: int) -> Affine:
    """rasterio 1.4.3 windows.transform(): translation of the window origin composed with the transform."""
    x, y = transform * ((col_off or 0.0), (row_off or 0.0))
    return Affine.translation(x - transform.c, y - transform.f) * transform


@dataclass
class GeoRaster:
    data: np.ndarray                 # (count, height, width)
    transform: Optional[Affine] = None
    epsg: Optional[int] = None
    nodata: Optional[float] = None
    extra_geokeys: dict = field(default_factory=dict)

    @property
    def count(self) -> int:
        return self.data.shape[0]

    @property
    def height(self) -> int:
        return self.data.shape[1]

    @property
    def width(self) -> int:
        return self.data.shape[2]

    @property
    def dtype(self) -> np.dtype:
        return self.data.dtype

    @property
    def crs_string(self) -> Optional[str]:
        """rasterio CRS.to_string() for EPSG-coded CRSs."""
        return f"EPSG:{self.epsg}" if self.epsg else None

    @property
    def bounds(self) -> Tuple[float, float, float, float]:
        """rasterio DatasetBase.bounds for north-up transforms: (left, bottom, right, top)."""
        return bounds_of(self.transform or Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0), self.width, self.height)


def bounds_of(t: Affine, width: int, height: int) -> Tuple[float, float, float, float]:
    """(left, bottom, right, top) of a width x height raster with transform t (rasterio DatasetBase.bounds)."""
    a, b, c, d, e, f = t.to_tuple()
    if b == d == 0:
        return (c, f + e * height, c + a * width, f)
    xs = [c, c + a * width, c + b * height, c + a * width + b * height]
    ys = [f, f + d * width, f + e * height, f + d * width + e * height]
    return (min(xs), min(ys), max(xs), max(ys))


def _lzw_decode(data: bytes) -> bytes:
    out = bytearray()
    table = [bytes([i]) for i in range(256)] + [b"", b""]
    bitpos, nbits, prev = 0, 9, None
    total = len(data) * 8
    while bitpos + nbits <= total:
        byte = bitpos >> 3
        chunk = int.from_bytes(data[byte:byte + 4].ljust(4, b"\0"), "big")
        code = (chunk >> (32 - nbits - (bitpos & 7))) & ((1 << nbits) - 1)
        bitpos += nbits
        if code == 256:
            table = table[:258]
            nbits, prev = 9, None
            continue
        if code == 257:
            break
        if prev is None:
            entry = table[code]
        elif code < len(table):
            entry = table[code]
            table.append(prev + entry[:1])
        else:
            entry = prev + prev[:1]
            table.append(entry)
        out += entry
        prev = entry
        if len(table) + 1 >= (1 << nbits) and nbits < 12:
            nbits += 1
    return bytes(out)


def _packbits_decode(data: bytes) -> bytes:
    out = bytearray()
    i = 0
    while i < len(data):
        n = data[i] if data[i] < 128 else data[i] - 256
        i += 1
        if n >= 0:
            out += data[i:i + n + 1]
            i += n + 1
        elif n != -128:
            out += data[i:i + 1] * (1 - n)
            i += 1
    return bytes(out)


class TiffFile:
    """A GeoTIFF opened by memory map: tags parsed once, pixel rows decoded on demand.

    ``read_rows(row0, row1, bands)`` decodes only the strips / tiles that intersect the rows (uncompressed chunks
    are viewed in place), so a rank of the sharded create-streaming reads its band-1 slab without touching the
    rest of the file -- the reference's per-tile ``src.read(1, window=...)`` (cli.py:698-699) at slab granularity.
    """

    def __init__(self, path):
        import mmap
        self.path = Path(path)
        self._f = open(self.path, "rb")
        size = self.path.stat().st_size
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
        buf = self._mm
        bo = "<" if buf[:2] == b"II" else ">"
        magic = struct.unpack(bo + "H", buf[2:4])[0]
        if magic == 42:
            off = struct.unpack(bo + "I", buf[4:8])[0]
            big = False
        elif magic == 43:
            off = struct.unpack(bo + "Q", buf[8:16])[0]
            big = True
        else:
            raise ValueError(f"{path}: not a TIFF")
        if big:
            n = struct.unpack(bo + "Q", buf[off:off + 8])[0]
            ent, esz, base = 20, 8, off + 8
        else:
            n = struct.unpack(bo + "H", buf[off:off + 2])[0]
            ent, esz, base = 12, 4, off + 2
        tags = {}
        for i in range(n):
            e = buf[base + ent * i: base + ent * (i + 1)]
            tag, typ = struct.unpack(bo + "HH", e[:4])
            cnt = struct.unpack(bo + ("Q" if big else "I"), e[4:4 + esz])[0]
            fmt, sz = _TYPES.get(typ, ("B", 1))
            nbytes = sz * cnt
            raw = e[4 + esz:4 + 2 * esz]
            if nbytes > esz:
                vo = struct.unpack(bo + ("Q" if big else "I"), raw)[0]
                raw = buf[vo:vo + nbytes]
            if typ == 2:
                tags[tag] = raw[:cnt].split(b"\0")[0].decode("latin-1")
            else:
                tags[tag] = struct.unpack(bo + fmt * cnt, raw[:nbytes])
        self.tags = tags
        self.width, self.height = tags[256][0], tags[257][0]
        self.spp = tags.get(277, (1,))[0]
        bits = tags.get(258, (8,))[0]
        sfmt = tags.get(339, (1,))[0]
        self.comp = tags.get(259, (1,))[0]
        self.planar = tags.get(284, (1,))[0]
        self.pred = tags.get(317, (1,))[0]
        kind = {1: "u", 2: "i", 3: "f"}[sfmt]
        self.file_dtype = np.dtype(f"{bo}{kind}{bits // 8}")
        self.dtype = self.file_dtype.newbyteorder("=")

    def close(self):
        if self._mm:
            try:
                self._mm.close()
            except BufferError:
                # numpy views of the map are still alive (e.g. held by an exception's traceback): leave the map to
                # the garbage collector rather than masking the caller's error with this one
                pass
            self._mm = None
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def count(self) -> int:
        return self.spp

    def _decomp(self, k: int, offs, cnts, nelem: int) -> np.ndarray:
        b = self._mm[offs[k]:offs[k] + cnts[k]] if self.comp != 1 else None
        if self.comp == 1:
            return np.frombuffer(self._mm, dtype=self.file_dtype, count=nelem, offset=offs[k])
        if self.comp in (8, 32946):
            raw = zlib.decompress(b)
        elif self.comp == 5:
            raw = _lzw_decode(b)
        elif self.comp == 32773:
            raw = _packbits_decode(b)
        else:
            raise NotImplementedError(f"TIFF compression {self.comp}")
        return np.frombuffer(raw, dtype=self.file_dtype)[:nelem]

    def read_rows(self, row0: int = 0, row1: Optional[int] = None, bands: Optional[List[int]] = None) -> np.ndarray:
        """Pixels of rows [row0, row1) of the given 0-based bands (default: all) -> (len(bands), rows, width)."""
        H, W, spp = self.height, self.width, self.spp
        row1 = H if row1 is None else min(row1, H)
        bands = list(range(spp)) if bands is None else list(bands)
        nr = max(0, row1 - row0)
        dt = self.file_dtype
        out = np.empty((len(bands), nr, W), dtype=self.dtype)
        if nr == 0:
            return out
        tags = self.tags
        chunky = self.planar != 2
        cs = spp if chunky else 1
        planes = [0] if chunky else bands  # planes to decode

        if 322 in tags:  # tiled
            tw, th = tags[322][0], tags[323][0]
            offs, cnts = tags[324], tags[325]
            tx, ty = (W + tw - 1) // tw, (H + th - 1) // th
            for pl in planes:
                sel = [(j, b) for j, b in enumerate(bands)] if chunky else [(bands.index(pl), 0)]
                for jt in range(row0 // th, (row1 - 1) // th + 1):
                    for i in range(tx):
                        k = pl * tx * ty + jt * tx + i
                        a = self._decomp(k, offs, cnts, th * tw * cs).reshape(th, tw, cs)
                        if self.pred == 2:
                            a = np.cumsum(a, axis=1, dtype=dt)
                        h, w = min(th, H - jt * th), min(tw, W - i * tw)
                        lo, hi = max(jt * th, row0), min(jt * th + h, row1)
                        for j, bsel in sel:
                            out[j, lo - row0:hi - row0, i * tw:i * tw + w] = a[lo - jt * th:hi - jt * th, :w, bsel]
        else:
            rps = tags.get(278, (H,))[0]
            offs, cnts = tags[273], tags[279]
            nstrips = (H + rps - 1) // rps
            for pl in planes:
                sel = [(j, b) for j, b in enumerate(bands)] if chunky else [(bands.index(pl), 0)]
                for sidx in range(row0 // rps, (row1 - 1) // rps + 1):
                    k = pl * nstrips + sidx
                    rows = min(rps, H - sidx * rps)
                    a = self._decomp(k, offs, cnts, rows * W * cs).reshape(rows, W, cs)
                    if self.pred == 2:
                        a = np.cumsum(a, axis=1, dtype=dt)
                    lo, hi = max(sidx * rps, row0), min(sidx * rps + rows, row1)
                    for j, bsel in sel:
                        out[j, lo - row0:hi - row0] = a[lo - sidx * rps:hi - sidx * rps, :, bsel]
        return out

    def band_view(self, band: int = 0) -> Optional[np.ndarray]:
        """Zero-copy (height, width) view of one band on the memory map, or None when the layout does not allow it
        (compressed, predictor, tiled, pixel-interleaved multi-band, non-native byte order, or strips that are not
        back to back in the file)."""
        tags = self.tags
        if self.comp != 1 or self.pred != 1 or 322 in tags or not self.file_dtype.isnative:
            return None
        if self.spp > 1 and self.planar != 2:
            return None
        H, W, isz = self.height, self.width, self.file_dtype.itemsize
        rps = tags.get(278, (H,))[0]
        offs, cnts = tags[273], tags[279]
        nstrips = (H + rps - 1) // rps
        k0 = band * nstrips
        if len(offs) < k0 + nstrips:
            return None
        for i in range(nstrips):
            rows = min(rps, H - i * rps)
            k = k0 + i
            if cnts[k] != rows * W * isz or (i and offs[k] != offs[k - 1] + cnts[k - 1]):
                return None
        if offs[k0] + H * W * isz > len(self._mm):
            return None
        return np.frombuffer(self._mm, dtype=self.file_dtype, count=H * W, offset=offs[k0]).reshape(H, W)

    def georef(self):
        """(transform, epsg, nodata, extra geokeys) with GDAL GTiff semantics (PixelIsArea default)."""
        tags = self.tags
        transform = None
        if 34264 in tags:
            m = tags[34264]
            transform = Affine(m[0], m[1], m[3], m[4], m[5], m[7])
        elif 33550 in tags and 33922 in tags:
            sx, sy = tags[33550][0], tags[33550][1]
            tp = tags[33922]
            transform = Affine(sx, 0.0, tp[3] - tp[0] * sx, 0.0, -sy, tp[4] + tp[1] * sy)
        epsg = None
        extra = {}
        if 34735 in tags:
            gk = tags[34735]
            nkeys = gk[3]
            raster_type = 1
            for i in range(nkeys):
                kid, loc, cnt, val = gk[4 + 4 * i: 8 + 4 * i]
                if loc == 0:
                    extra[kid] = val
                    if kid in (3072, 2048) and val not in (0, 32767):
                        epsg = int(val) if (kid == 3072 or epsg is None) else epsg
                    if kid == 1025:
                        raster_type = val
            if raster_type == 2 and transform is not None and 34264 not in tags:
                # PixelIsPoint: GDAL shifts the origin by half a pixel (GTIFF_POINT_GEO_IGNORE=FALSE)
                transform = Affine(transform.a, transform.b, transform.c - 0.5 * transform.a - 0.5 * transform.b,
                                   transform.d, transform.e, transform.f - 0.5 * transform.d - 0.5 * transform.e)
        nodata = None
        if 42113 in tags:
            try:
                nodata = float(tags[42113])
            except ValueError:
                nodata = None
        return transform, epsg, nodata, extra

    def raster(self, row0: int = 0, row1: Optional[int] = None, bands: Optional[List[int]] = None) -> GeoRaster:
        transform, epsg, nodata, extra = self.georef()
        return GeoRaster(data=self.read_rows(row0, row1, bands), transform=transform, epsg=epsg, nodata=nodata,
                         extra_geokeys=extra)


def read(path) -> GeoRaster:
    """The whole raster (rasterio ``src.read()``)."""
    with TiffFile(path) as tf:
        return tf.raster()


def write(path, data: np.ndarray, transform: Optional[Affine] = None, epsg: Optional[int] = None,
          nodata: Optional[float] = None, compress: Optional[str] = None, predictor: int = 1,
          tile: Optional[int] = None, planar: int = 1, rows_per_strip: Optional[int] = None) -> None:
    """Write (count, height, width) GTiff (GDAL-like layout): ~8 KB strips by default (or `rows_per_strip` rows), or
    `tile` x `tile` tiles; chunky (planar 1) or band-sequential (planar 2) samples; uncompressed or
    ``compress="deflate"`` with optional horizontal differencing (predictor 2).  Uncompressed strips are written
    straight from the array (no staging copy: a multi-GB raster streams to the file)."""
    a = np.asarray(data)
    if a.ndim == 2:
        a = a[None]
    count, H, W = a.shape
    dt = a.dtype
    a = np.ascontiguousarray(a.astype(dt.newbyteorder("<"), copy=False))
    chunky = planar == 1 or count == 1
    cs = count if chunky else 1
    planes = [np.ascontiguousarray(a.transpose(1, 2, 0))] if chunky else [a[b][:, :, None] for b in range(count)]

    def encode_chunk(x: np.ndarray) -> bytes:  # x: (rows, cols, cs)
        if predictor == 2:
            x = x.copy()
            x[:, 1:] = np.diff(x, axis=1)
        b = np.ascontiguousarray(x).tobytes()
        return zlib.compress(b, 6) if compress == "deflate" else b

    chunks: List[bytes] = []
    direct = not tile and compress is None and predictor != 2  # strips written from array views
    strips: List[np.ndarray] = []
    if tile:
        tw = th = int(tile)
        tx, ty = (W + tw - 1) // tw, (H + th - 1) // th
        for pl in planes:
            for j in range(ty):
                for i in range(tx):
                    blk = np.zeros((th, tw, cs), dtype=a.dtype)
                    src = pl[j * th:(j + 1) * th, i * tw:(i + 1) * tw]
                    blk[:src.shape[0], :src.shape[1]] = src
                    chunks.append(encode_chunk(blk))
        rps = None
    else:
        row_bytes = W * cs * dt.itemsize
        rps = int(rows_per_strip) if rows_per_strip else max(1, min(H, 8192 // max(1, row_bytes)))
        rps = max(1, min(H, rps))
        nstrips = (H + rps - 1) // rps
        for pl in planes:
            for st in range(nstrips):
                if direct:
                    strips.append(pl[st * rps:(st + 1) * rps])
                else:
                    chunks.append(encode_chunk(pl[st * rps:(st + 1) * rps]))
    sizes = [x.size * dt.itemsize for x in strips] if direct else [len(c) for c in chunks]
    total = sum(sizes)
    big = total > 0xF0000000
    sfmt = 3 if dt.kind == "f" else (2 if dt.kind == "i" else 1)
    entries: List[Tuple[int, int, tuple]] = []

    def add(tag, typ, vals):
        entries.append((tag, typ, tuple(vals) if isinstance(vals, (list, tuple)) else (vals,)))

    off_tag, cnt_tag = (324, 325) if tile else (273, 279)
    add(256, 3 if W < 65536 else 4, W)
    add(257, 3 if H < 65536 else 4, H)
    add(258, 3, [dt.itemsize * 8] * count)
    add(259, 3, 8 if compress == "deflate" else 1)
    add(262, 3, 2 if (count == 3 and dt == np.uint8) else 1)
    if not tile:
        add(273, 16 if big else 4, [0] * len(sizes))  # patched below
    add(277, 3, count)
    if not tile:
        add(278, 3 if rps < 65536 else 4, rps)
        add(279, 16 if big else 4, sizes)
    add(284, 3, 1 if chunky else 2)
    if predictor == 2:
        add(317, 3, 2)
    if tile:
        add(322, 3, int(tile))
        add(323, 3, int(tile))
        add(324, 16 if big else 4, [0] * len(chunks))  # patched below
        add(325, 16 if big else 4, [len(c) for c in chunks])
    if count > 1 and not (count == 3 and dt == np.uint8):
        add(338, 3, [0] * (count - 1))
    add(339, 3, [sfmt] * count)
    if transform is not None:
        t = transform
        if t.b == 0 and t.d == 0:
            add(33550, 12, [t.a, -t.e, 0.0])
            add(33922, 12, [0.0, 0.0, 0.0, t.c, t.f, 0.0])
        else:
            add(34264, 12, [t.a, t.b, 0.0, t.c, t.d, t.e, 0.0, t.f, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0])
    if epsg:
        geographic = epsg in (4326, 4269, 4258, 4267) or 4000 <= epsg < 5000
        keys = [(1024, 0, 1, 2 if geographic else 1), (1025, 0, 1, 1),
                (2048 if geographic else 3072, 0, 1, int(epsg))]
        gk = [1, 1, 0, len(keys)]
        for k in keys:
            gk += list(k)
        add(34735, 3, gk)
    if nodata is not None:
        add(42113, 2, (repr(float(nodata)) if float(nodata) != int(nodata) else str(int(nodata))).encode() + b"\0")
    entries.sort(key=lambda x: x[0])

    # layout: header | IFD | out-of-line values | pixel data
    hdr = 16 if big else 8
    ent = 20 if big else 12
    ifd_size = (8 + len(entries) * ent + 8) if big else (2 + len(entries) * ent + 4)
    esz = 8 if big else 4
    ool_base = hdr + ifd_size
    chunk_off = np.zeros(len(sizes) + 1, dtype=np.int64)
    chunk_off[1:] = np.cumsum(sizes)

    def pack_vals(typ, vals):
        if typ == 2:
            return bytes(vals[0]) if isinstance(vals[0], (bytes, bytearray)) else bytes(vals)
        fmt, _ = _TYPES[typ]
        return struct.pack("<" + fmt * len(vals), *vals)

    # pixel data offset depends on the out-of-line size: two passes
    def build(data_off):
        out_ool = bytearray()
        ifd = bytearray()
        ifd += struct.pack("<Q", len(entries)) if big else struct.pack("<H", len(entries))
        for tag, typ, vals in entries:
            if tag == off_tag:
                vals = tuple(int(data_off + o) for o in chunk_off[:-1])
            payload = pack_vals(typ, vals)
            cnt = len(payload) if typ == 2 else len(vals)
            ifd += struct.pack("<HH", tag, typ) + (struct.pack("<Q", cnt) if big else struct.pack("<I", cnt))
            if len(payload) <= esz:
                ifd += payload.ljust(esz, b"\0")
            else:
                off = ool_base + len(out_ool)
                ifd += struct.pack("<Q", off) if big else struct.pack("<I", off)
                out_ool += payload
                if len(out_ool) % 2:
                    out_ool += b"\0"
        ifd += struct.pack("<Q", 0) if big else struct.pack("<I", 0)
        return ifd, out_ool

    _, ool = build(0)
    data_off = ool_base + len(ool)
    ifd, ool = build(data_off)
    with open(path, "wb") as fh:
        if big:
            fh.write(b"II" + struct.pack("<HHHQ", 43, 8, 0, hdr))
        else:
            fh.write(b"II" + struct.pack("<HI", 42, hdr))
        fh.write(ifd)
        fh.write(ool)
        for c in chunks:
            fh.write(c)
        for x in strips:
            fh.write(memoryview(np.ascontiguousarray(x)).cast("B"))
