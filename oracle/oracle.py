"""oracle.oracle -- TEST INFRASTRUCTURE ONLY: ctypes bindings to the CPU oracle (flac_oracle.c).

The oracle restates the reference's hot path on the CPU (see flac_oracle.c header for the
reference file:line each function follows).  Only tests/, __graft_entry__.smoke() and bench.py's
``cpu_baseline`` leg may import this module; the product (flac_raster_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "liborc_flac.so"
_lib = None

# dtype codes (shared numbering with include/flac_raster_amd.h FRS_DT_*)
DTYPES = {np.dtype(np.uint8): 1, np.dtype(np.uint16): 2, np.dtype(np.int16): 3,
          np.dtype(np.int32): 4, np.dtype(np.uint32): 5, np.dtype(np.float32): 6,
          np.dtype(np.float64): 7}


def build(force: bool = False) -> Path:
    """Compile flac_oracle.c into liborc_flac.so with the committed Makefile."""
    if force or not _LIB_PATH.exists() or _LIB_PATH.stat().st_mtime < (_HERE / "flac_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(_HERE), "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(_LIB_PATH))
        i64, i32, vp, dp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
        L.orc_encode_frames.restype = i64
        L.orc_encode_frames.argtypes = [vp, i64, i32, i32, i32, i32, vp, i64]
        L.orc_encode_frames_level.restype = i64
        L.orc_encode_frames_level.argtypes = [vp, i64, i32, i32, i32, i32, i32, vp, i64]
        L.orc_stream_header.restype = i64
        L.orc_stream_header.argtypes = [i32, i32, i32, i32, vp, i64]
        L.orc_normalize.restype = i32
        L.orc_normalize.argtypes = [vp, i32, i64, i32, dp, dp, vp]
        L.orc_denormalize_i16.restype = None
        L.orc_denormalize_i16.argtypes = [vp, i64, i32, ctypes.c_double, ctypes.c_double, i32, vp]
        L.orc_decode_frames.restype = i64
        L.orc_decode_frames.argtypes = [vp, i64, i32, i32, vp, i64]
        L.orc_decode_frames_ca.restype = i64
        L.orc_decode_frames_ca.argtypes = [vp, i64, i32, i32, vp, i64, vp, i64]
        L.orc_decode_frames_sf.restype = i64
        L.orc_decode_frames_sf.argtypes = [vp, i64, i32, i32, vp, i64, vp, i64]
        L.orc_encode_tiles.restype = i64
        L.orc_encode_tiles.argtypes = [vp, i32, i64, i64, i64, i32, i32, i32, vp, i64, vp, vp, vp, i32]
        L.orc_normalize_spatial.restype = i32
        L.orc_normalize_spatial.argtypes = [vp, i32, i64, vp]
        L.orc_window_tukey.restype = None
        L.orc_window_tukey.argtypes = [vp, i32, ctypes.c_float]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def bits_per_sample_for(dtype) -> int:
    """converter.py:25-37 (_calculate_audio_params, bit depth part)."""
    dt = np.dtype(dtype)
    if dt in (np.uint8, np.uint16, np.int16):
        return 16
    return 24


def sample_rate_for(shape0: int, shape1: int) -> int:
    """converter.py:39-51 -- total_pixels = shape[0]*shape[1] of the (bands, h, w) array."""
    total = shape0 * shape1
    if total < 1000000:
        return 44100
    if total < 10000000:
        return 48000
    if total < 100000000:
        return 96000
    return 192000


def normalize(arr: np.ndarray):
    """converter.py:56-86 -> (pcm int32 array same shape, data_min, data_max, stream_bps)."""
    a = np.ascontiguousarray(arr)
    out = np.empty(a.shape, dtype=np.int32)
    mn, mx = ctypes.c_double(), ctypes.c_double()
    bps = lib().orc_normalize(_ptr(a), DTYPES[a.dtype], a.size, bits_per_sample_for(a.dtype),
                              ctypes.byref(mn), ctypes.byref(mx), _ptr(out))
    return out, mn.value, mx.value, bps


def normalize_spatial(arr: np.ndarray) -> np.ndarray:
    """spatial_encoder.py:229-248 + pyflac's astype(int32): samples in {-1, 0, 1}."""
    a = np.ascontiguousarray(arr)
    out = np.empty(a.shape, dtype=np.int32)
    if lib().orc_normalize_spatial(_ptr(a), DTYPES[a.dtype], a.size, _ptr(out)) != 0:
        raise ValueError("pyflac rejects the 64-bit sample array of this dtype")
    return out


def encode_frames(pcm: np.ndarray, bps: int, sample_rate: int, blocksize: int = 4096, level: int = 5) -> bytes:
    """libFLAC frames at compression `level` (0..8) for interleaved pcm [N, C] (levels 6..8 and loose mid/side at
    levels 1 / 4 on two channels: restated, parity unpinned -- oracle/flac_oracle.c decide_subframe)."""
    x = np.ascontiguousarray(pcm, dtype=np.int32)
    if x.ndim == 1:
        x = x[:, None]
    n, c = x.shape
    cap = n * c * (bps // 8 + 1) + (n // blocksize + 2) * (32 + 16 * c) + 1024
    out = np.empty(cap, dtype=np.uint8)
    r = lib().orc_encode_frames_level(_ptr(x), n, c, bps, sample_rate, blocksize, level, _ptr(out), cap)
    if r == -2:
        raise ValueError(f"compression level {level} with {c} channels is not restated")
    if r < 0:
        raise RuntimeError(f"oracle encode overflow {r}")
    return out[:r].tobytes()


def stream_header(channels: int, bps: int, sample_rate: int, blocksize: int = 4096) -> bytes:
    out = np.empty(128, dtype=np.uint8)
    r = lib().orc_stream_header(channels, bps, sample_rate, blocksize, _ptr(out), 128)
    return out[:r].tobytes()


def decode_frames(data: bytes, channels: int, bps: int, max_samples: int) -> np.ndarray:
    buf = np.frombuffer(data, dtype=np.uint8)
    out = np.empty((max_samples, channels), dtype=np.int32)
    r = lib().orc_decode_frames(_ptr(buf), len(buf), channels, bps, _ptr(out), max_samples)
    if r < 0:
        raise RuntimeError(f"oracle decode error {r}")
    return out[:r]


def frame_assignments(data: bytes, channels: int, bps: int, max_samples: int) -> np.ndarray:
    """Channel-assignment code of every frame (0..7 independent, 8 left-side, 9 right-side, 10 mid-side)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    out = np.empty((max_samples, channels), dtype=np.int32)
    ca = np.empty(max_samples // 16 + 16, dtype=np.int8)
    r = lib().orc_decode_frames_ca(_ptr(buf), len(buf), channels, bps, _ptr(out), max_samples, _ptr(ca), len(ca))
    if r < 0:
        raise RuntimeError(f"oracle decode error {r}")
    return ca[: -(-r // 4096) if r else 0].copy()


def subframe_types(data: bytes, channels: int, bps: int, max_samples: int) -> np.ndarray:
    """(type code, residual partition order) of every subframe, frame-major: type 0 CONSTANT, 1 VERBATIM,
    8 + order FIXED, 31 + order LPC; partition order -1 for CONSTANT / VERBATIM."""
    buf = np.frombuffer(data, dtype=np.uint8)
    out = np.empty((max_samples, channels), dtype=np.int32)
    cap = (max_samples // 16 + 16) * channels
    sf = np.full(cap, -1, dtype=np.int16)
    r = lib().orc_decode_frames_sf(_ptr(buf), len(buf), channels, bps, _ptr(out), max_samples, _ptr(sf), cap)
    if r < 0:
        raise RuntimeError(f"oracle decode error {r}")
    sf = sf[: (-(-r // 4096) if r else 0) * channels]
    t = sf & 0xFF
    po = np.where((t >= 8), sf >> 8, -1)
    return np.stack([t, po], axis=1)


def denormalize_i16(pcm: np.ndarray, dmin: float, dmax: float, dtype, pcm_bps: int = 16) -> np.ndarray:
    """converter.py:88-110 after pyflac+soundfile's PCM_16 WAV round trip (sonos-pyflac.txt:1629)."""
    p = np.ascontiguousarray(pcm, dtype=np.int32)
    out = np.empty(p.shape, dtype=dtype)
    lib().orc_denormalize_i16(_ptr(p), p.size, pcm_bps, dmin, dmax, DTYPES[np.dtype(dtype)], _ptr(out))
    return out


def window_tukey(L: int, p: float = 0.5) -> np.ndarray:
    w = np.empty(L, dtype=np.float32)
    lib().orc_window_tukey(_ptr(w), L, p)
    return w


def encode_tiles(band: np.ndarray, tile: int, sample_rate: int = 44100, blocksize: int = 4096, threads: int = 1):
    """Band-1 streaming tiles (cli.py:690-763): returns (arena bytes, tile_off, mins, maxs)."""
    b = np.ascontiguousarray(band)
    H, W = b.shape
    nt = ((H + tile - 1) // tile) * ((W + tile - 1) // tile)
    esz = b.dtype.itemsize
    cap = H * W * (4 if esz <= 2 else 5) + nt * 4096 + 4096
    arena = np.empty(cap, dtype=np.uint8)
    off = np.zeros(nt + 1, dtype=np.int64)
    mins = np.zeros(nt, dtype=np.float64)
    maxs = np.zeros(nt, dtype=np.float64)
    r = lib().orc_encode_tiles(_ptr(b), DTYPES[b.dtype], H, W, W, tile, sample_rate, blocksize,
                               _ptr(arena), cap, _ptr(off), _ptr(mins), _ptr(maxs), threads)
    if r < 0:
        raise RuntimeError(f"oracle encode_tiles failed {r}")
    return arena[:r], off, mins, maxs
