#!/usr/bin/env python3
"""Round 6 measurement: which subframe types libFLAC level 5 picks on the C4 workload (GPU-encoded, byte-equal to the
oracle), from the frame headers of the first tiles' frames.  Decides whether keeping the LPC residuals for the
packing pass (and re-loading the samples when FIXED or VERBATIM wins) pays.
usage: python tools/r6/subframe_types.py [tiles]   (one JSON line)"""
import json
import sys
from collections import Counter
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from flac_raster_amd import _native  # noqa: E402

CRC8 = []
for i in range(256):
    c = i
    for _ in range(8):
        c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    CRC8.append(c)


def crc8(b):
    c = 0
    for x in b:
        c = CRC8[c ^ x]
    return c


def header_len(buf, p):
    """length of a frame header at p (its CRC-8 checked), or 0"""
    if p + 6 > len(buf) or buf[p] != 0xFF or (buf[p + 1] & 0xFE) != 0xF8:
        return 0
    bsc, src = buf[p + 2] >> 4, buf[p + 2] & 15
    q = p + 4
    b0 = buf[q]
    n = 1 if b0 < 0x80 else 2 if b0 >= 0xC0 and b0 < 0xE0 else 3 if b0 < 0xF0 else 4 if b0 < 0xF8 else 5
    q += n
    q += 1 if bsc == 6 else 2 if bsc == 7 else 0
    q += 1 if src == 12 else 2 if src in (13, 14) else 0
    if q >= len(buf) or crc8(buf[p:q]) != buf[q]:
        return 0
    return q + 1 - p


def main():
    ntiles = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    H = W = 40000
    B, T = 4, 512
    ctx = _native.Context(0)
    raster = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(raster, B, H, W, row0=0, full_height=H, seed=1234)
    desc = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena)
    ctx.sync()
    types = Counter()
    orders = Counter()
    pords = Counter()
    step = max(1, (len(off) - 1) // ntiles)
    for t in range(0, len(off) - 1, step):
        buf = arena.download(int(off[t + 1] - off[t]), int(off[t])).tobytes()
        p = 0
        while p < len(buf):
            h = header_len(buf, p)
            if h:
                st = buf[p + h] >> 1 & 0x3F
                kind = "CONSTANT" if st == 0 else "VERBATIM" if st == 1 else "FIXED" if 8 <= st <= 12 else \
                    "LPC" if st >= 32 else "other"
                types[kind] += 1
                orders[f"{kind}{(st - 8) if kind == 'FIXED' else (st - 31) if kind == 'LPC' else ''}"] += 1
                if kind in ("FIXED", "LPC"):  # the residual's partition order (16-bit stream, no wasted bits)
                    o = (st - 8) if kind == "FIXED" else (st - 31)
                    v = int.from_bytes(buf[p + h:p + h + 64], "big")
                    nb = 64 * 8
                    pos = 8 + (buf[p + h] & 1)  # (a wasted-bits flag would add a unary count: C4 has none)
                    pos += o * 16
                    if kind == "LPC":
                        prec = ((v >> (nb - pos - 4)) & 15) + 1
                        pos += 4 + 5 + o * prec
                    pos += 2
                    po = (v >> (nb - pos - 4)) & 15
                    pords[f"{kind}-po{po}"] += 1
                p += h + 1000  # (frames are > 1 KB: skip ahead, then find the next sync)
            else:
                p += 1
    print(json.dumps({"tiles": len(range(0, len(off) - 1, step)), "types": dict(types), "orders": dict(orders), "partition_orders": dict(pords)}),
          flush=True)


if __name__ == "__main__":
    main()
