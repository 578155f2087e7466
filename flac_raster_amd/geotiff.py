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


def read(path) -> GeoRaster:
    buf = Path(path).read_bytes()
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
    W, H = tags[256][0], tags[257][0]
    spp = tags.get(277, (1,))[0]
    bits = tags.get(258, (8,))[0]
    sfmt = tags.get(339, (1,))[0]
    comp = tags.get(259, (1,))[0]
    planar = tags.get(284, (1,))[0]
    pred = tags.get(317, (1,))[0]
    kind = {1: "u", 2: "i", 3: "f"}[sfmt]
    dt = np.dtype(f"{bo}{kind}{bits // 8}")

    def decomp(b: bytes) -> bytes:
        if comp == 1:
            return b
        if comp in (8, 32946):
            return zlib.decompress(b)
        if comp == 5:
            return _lzw_decode(b)
        if comp == 32773:
            return _packbits_decode(b)
        raise NotImplementedError(f"TIFF compression {comp}")

    nplanes = spp if planar == 2 else 1
    cs = 1 if planar == 2 else spp
    out = np.zeros((nplanes, H, W, cs), dtype=dt)
    if 322 in tags:  # tiled
        tw, th = tags[322][0], tags[323][0]
        offs, cnts = tags[324], tags[325]
        tx = (W + tw - 1) // tw
        ty = (H + th - 1) // th
        for pl in range(nplanes):
            for j in range(ty):
                for i in range(tx):
                    k = pl * tx * ty + j * tx + i
                    a = np.frombuffer(decomp(buf[offs[k]:offs[k] + cnts[k]]), dtype=dt)[:th * tw * cs]
                    a = a.reshape(th, tw, cs)
                    if pred == 2:
                        a = np.cumsum(a, axis=1, dtype=dt)
                    h = min(th, H - j * th)
                    w = min(tw, W - i * tw)
                    out[pl, j * th:j * th + h, i * tw:i * tw + w] = a[:h, :w]
    else:
        rps = tags.get(278, (H,))[0]
        offs, cnts = tags[273], tags[279]
        nstrips = (H + rps - 1) // rps
        for pl in range(nplanes):
            for s in range(nstrips):
                k = pl * nstrips + s
                rows = min(rps, H - s * rps)
                a = np.frombuffer(decomp(buf[offs[k]:offs[k] + cnts[k]]), dtype=dt)[:rows * W * cs]
                a = a.reshape(rows, W, cs)
                if pred == 2:
                    a = np.cumsum(a, axis=1, dtype=dt)
                out[pl, s * rps:s * rps + rows] = a
    if planar == 2:
        data = out[:, :, :, 0]
    else:
        data = out[0].transpose(2, 0, 1)
    data = np.ascontiguousarray(data).astype(dt.newbyteorder("="), copy=False)
    # georeferencing (GDAL GTiff semantics, PixelIsArea default)
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
    return GeoRaster(data=data, transform=transform, epsg=epsg, nodata=nodata, extra_geokeys=extra)


def write(path, data: np.ndarray, transform: Optional[Affine] = None, epsg: Optional[int] = None,
          nodata: Optional[float] = None) -> None:
    """Write (count, height, width) uncompressed GTiff (GDAL-like layout)."""
    a = np.asarray(data)
    if a.ndim == 2:
        a = a[None]
    count, H, W = a.shape
    dt = a.dtype
    a = np.ascontiguousarray(a.astype(dt.newbyteorder("<"), copy=False))
    pix = np.ascontiguousarray(a.transpose(1, 2, 0)) if count > 1 else a[0]
    row_bytes = W * count * dt.itemsize
    rps = max(1, min(H, 8192 // max(1, row_bytes)))
    nstrips = (H + rps - 1) // rps
    raw = pix.tobytes()
    big = len(raw) > 0xF0000000
    sfmt = 3 if dt.kind == "f" else (2 if dt.kind == "i" else 1)
    entries: List[Tuple[int, int, tuple]] = []

    def add(tag, typ, vals):
        entries.append((tag, typ, tuple(vals) if isinstance(vals, (list, tuple)) else (vals,)))

    add(256, 3 if W < 65536 else 4, W)
    add(257, 3 if H < 65536 else 4, H)
    add(258, 3, [dt.itemsize * 8] * count)
    add(259, 3, 1)
    add(262, 3, 2 if (count == 3 and dt == np.uint8) else 1)
    add(273, 16 if big else 4, [0] * nstrips)  # patched below
    add(277, 3, count)
    add(278, 3 if rps < 65536 else 4, rps)
    add(279, 16 if big else 4, [min(rps, H - s * rps) * row_bytes for s in range(nstrips)])
    add(284, 3, 1)
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
    ool = bytearray()
    ool_base = hdr + ifd_size

    def pack_vals(typ, vals):
        if typ == 2:
            return bytes(vals[0]) if isinstance(vals[0], (bytes, bytearray)) else bytes(vals)
        fmt, _ = _TYPES[typ]
        return struct.pack("<" + fmt * len(vals), *vals)

    # pixel data offset depends on ool size: compute two passes
    def build(data_off):
        out_ool = bytearray()
        ifd = bytearray()
        ifd += struct.pack("<Q", len(entries)) if big else struct.pack("<H", len(entries))
        for tag, typ, vals in entries:
            if tag == 273:
                vals = tuple(data_off + s * rps * row_bytes for s in range(nstrips))
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
        fh.write(raw)
