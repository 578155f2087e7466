"""ctypes binding of libflac_raster_amd.so (C-ABI declared in include/flac_raster_amd.h).

There is deliberately no CPU fallback: if the library is not built, or there is no gfx950 device, every
codec entry point raises :class:`NativeUnavailable`.  The CPU oracle under ``oracle/`` is test
infrastructure and is never imported here.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from pathlib import Path
from typing import Optional, Sequence, Tuple

import numpy as np

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libflac_raster_amd.so"

FRS_OK = 0
STATUS = {-1: "FRS_E_ARG", -2: "FRS_E_HIP", -3: "FRS_E_NOSPACE", -4: "FRS_E_CORRUPT",
          -5: "FRS_E_UNSUPPORTED", -6: "FRS_E_NODEV"}

DTYPE_CODES = {np.dtype(np.uint8): 1, np.dtype(np.uint16): 2, np.dtype(np.int16): 3,
               np.dtype(np.int32): 4, np.dtype(np.uint32): 5, np.dtype(np.float32): 6,
               np.dtype(np.float64): 7}
_DT_CACHE = {}  # dtype argument -> (itemsize, DTYPE_CODES code): the bbox-query path skips np.dtype per call

# names every build must export (tests check them against include/flac_raster_amd.h)
EXPORTS = (
    "frs_abi_version", "frs_device_count", "frs_ctx_create", "frs_ctx_destroy", "frs_last_error",
    "frs_encode_arena_bound", "frs_encode_tiles_device", "frs_encode_tiles",
    "frs_decode_frames_device", "frs_decode_frames", "frs_decode_tiles_device", "frs_decode_tiles",
    "frs_decode_tile_device",
    "frs_denormalize_device", "frs_denormalize",
    "frs_dev_malloc", "frs_dev_free", "frs_host_malloc", "frs_host_free", "frs_memcpy_h2d", "frs_memcpy_d2h", "frs_ctx_sync",
    "frs_synth_raster_device", "frs_ctx_stream", "frs_profile_enable", "frs_profile_avg_ms",
    "frs_profile_reset", "frs_comm_unique_id", "frs_comm_init", "frs_comm_destroy", "frs_comm_allgather_i64",
)


class NativeUnavailable(RuntimeError):
    """The HIP library or a gfx950 device is missing (no CPU fallback exists)."""


class FrsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class EncodeDesc(ctypes.Structure):
    """frs_encode_desc"""
    _fields_ = [
        ("height", ctypes.c_int64), ("width", ctypes.c_int64),
        ("row_stride", ctypes.c_int64), ("band_stride", ctypes.c_int64),
        ("dtype", ctypes.c_int32), ("band0", ctypes.c_int32), ("nbands", ctypes.c_int32),
        ("tile_h", ctypes.c_int32), ("tile_w", ctypes.c_int32),
        ("blocksize", ctypes.c_int32), ("sample_rate", ctypes.c_int32),
        ("bits_per_sample", ctypes.c_int32), ("compression_level", ctypes.c_int32),
        ("norm_mode", ctypes.c_int32),
        ("tile_begin", ctypes.c_int64), ("tile_end", ctypes.c_int64),
    ]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: Optional[os.PathLike] = None):
    """Load (once) and prototype the shared library.  Raises NativeUnavailable if it is not built."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        # FRS_LIB_PATH: an alternative build of the same library (A/B experiments on one GPU box)
        p = Path(path) if path else Path(os.environ.get("FRS_LIB_PATH", str(LIB_PATH)))
        if not p.exists():
            raise NativeUnavailable(
                f"{p} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(str(p))
        i64, i32, vp, dp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
        ip64 = ctypes.POINTER(ctypes.c_int64)
        ctxp = ctypes.c_void_p
        L.frs_abi_version.restype = i32
        L.frs_abi_version.argtypes = []
        L.frs_device_count.restype = i32
        L.frs_device_count.argtypes = []
        L.frs_ctx_create.restype = i32
        L.frs_ctx_create.argtypes = [i32, ctypes.POINTER(ctxp)]
        L.frs_ctx_destroy.restype = None
        L.frs_ctx_destroy.argtypes = [ctxp]
        L.frs_last_error.restype = ctypes.c_char_p
        L.frs_last_error.argtypes = [ctxp]
        L.frs_encode_arena_bound.restype = i64
        L.frs_encode_arena_bound.argtypes = [ctypes.POINTER(EncodeDesc)]
        enc_args = [ctxp, ctypes.POINTER(EncodeDesc), vp, vp, i64, ip64, dp, dp, ctypes.POINTER(i32)]
        L.frs_encode_tiles_device.restype = i32
        L.frs_encode_tiles_device.argtypes = enc_args
        L.frs_encode_tiles.restype = i32
        L.frs_encode_tiles.argtypes = enc_args
        dec_args = [ctxp, vp, ip64, i32, i32, i32, i32, vp, ip64]
        L.frs_decode_frames_device.restype = i32
        L.frs_decode_frames_device.argtypes = dec_args
        L.frs_decode_frames.restype = i32
        L.frs_decode_frames.argtypes = dec_args
        dect_args = [ctxp, vp, ip64, i32, i32, i32, i32, ip64, dp, dp, i32, vp]
        L.frs_decode_tiles_device.restype = i32
        L.frs_decode_tiles_device.argtypes = dect_args
        L.frs_decode_tiles.restype = i32
        L.frs_decode_tiles.argtypes = dect_args
        L.frs_decode_tile_device.restype = i32
        L.frs_decode_tile_device.argtypes = [ctxp, vp, i64, i64, i64, i32, i32, i32, ctypes.c_double, ctypes.c_double,
                                             i32, vp]
        den_args = [ctxp, vp, i64, i32, ctypes.c_double, ctypes.c_double, i32, vp]
        L.frs_denormalize_device.restype = i32
        L.frs_denormalize_device.argtypes = den_args
        L.frs_denormalize.restype = i32
        L.frs_denormalize.argtypes = den_args
        L.frs_dev_malloc.restype = vp
        L.frs_dev_malloc.argtypes = [ctxp, i64]
        L.frs_dev_free.restype = None
        L.frs_dev_free.argtypes = [ctxp, vp]
        L.frs_host_malloc.restype = vp
        L.frs_host_malloc.argtypes = [ctxp, i64]
        L.frs_host_free.restype = None
        L.frs_host_free.argtypes = [ctxp, vp]
        L.frs_memcpy_h2d.restype = i32
        L.frs_memcpy_h2d.argtypes = [ctxp, vp, vp, i64]
        L.frs_memcpy_d2h.restype = i32
        L.frs_memcpy_d2h.argtypes = [ctxp, vp, vp, i64]
        L.frs_ctx_sync.restype = i32
        L.frs_ctx_sync.argtypes = [ctxp]
        L.frs_synth_raster_device.restype = i32
        L.frs_synth_raster_device.argtypes = [ctxp, vp, i32, i64, i64, i64, i64, ctypes.c_uint64]
        L.frs_ctx_stream.restype = vp
        L.frs_ctx_stream.argtypes = [ctxp]
        L.frs_profile_enable.restype = i32
        L.frs_profile_enable.argtypes = [ctxp, i32]
        L.frs_profile_avg_ms.restype = ctypes.c_double
        L.frs_profile_avg_ms.argtypes = [ctxp, ctypes.c_char_p]
        L.frs_profile_reset.restype = None
        L.frs_profile_reset.argtypes = [ctxp]
        L.frs_comm_unique_id.restype = i32
        L.frs_comm_unique_id.argtypes = [vp]
        L.frs_comm_init.restype = i32
        L.frs_comm_init.argtypes = [ctxp, vp, i32, i32, ctypes.POINTER(ctypes.c_void_p)]
        L.frs_comm_destroy.restype = None
        L.frs_comm_destroy.argtypes = [vp]
        L.frs_comm_allgather_i64.restype = i32
        L.frs_comm_allgather_i64.argtypes = [vp, ip64, i64, ip64]
        if L.frs_abi_version() != 1:
            raise NativeUnavailable("ABI version mismatch")
        if path is None:
            _lib = L
        return L


def device_count() -> int:
    return load_library().frs_device_count()


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _is_window_of(raster, desc) -> bool:
    """True when `raster` is a strided numpy view ([bands][rows][cols] or [rows][cols]) whose element strides are the
    descriptor's row_stride / band_stride: a window of a larger raster (cli.py:698-699, rasterio Window reads), passed
    to the C-ABI by its origin pointer without a contiguous copy."""
    if not isinstance(raster, np.ndarray) or raster.flags.c_contiguous or raster.ndim not in (2, 3):
        return False
    es = raster.dtype.itemsize
    st = raster.strides
    if st[-1] != es or any(x <= 0 or x % es for x in st):
        return False
    if st[-2] // es != desc.row_stride or raster.shape[-1] != desc.width or raster.shape[-2] != desc.height:
        return False
    return raster.ndim == 2 or (st[0] // es == desc.band_stride and raster.shape[0] >= desc.band0 + desc.nbands)


class DeviceBuffer:
    """A device allocation owned by a Context (freed with it or on close())."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        self.ptr = ctx.lib.frs_dev_malloc(ctx.handle, self.nbytes)
        if not self.ptr:
            raise FrsError(-2, ctx.last_error() or "device allocation failed")

    def upload(self, host: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(host)
        if offset + a.nbytes > self.nbytes:
            raise ValueError("upload exceeds buffer")
        self.ctx._check(self.ctx.lib.frs_memcpy_h2d(self.ctx.handle, self.ptr + offset, _p(a), a.nbytes))

    def download(self, nbytes: Optional[int] = None, offset: int = 0, out: Optional[np.ndarray] = None) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        dst = out if out is not None else np.empty(n, dtype=np.uint8)
        self.ctx._check(self.ctx.lib.frs_memcpy_d2h(self.ctx.handle, _p(dst), self.ptr + offset, n))
        return dst

    def close(self):
        if self.ptr:
            self.ctx.lib.frs_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory (frs_host_malloc) the device can address: a decode target the kernels store straight
    into (no device buffer, no D2H copy).  `array` is its uint8 view; freed with close()."""

    def __init__(self, ctx: "Context", nbytes: int):
        # a weak reference: the context caches one HostBuffer (Context._pin), and a strong one would make a cycle that
        # keeps a dropped context's streams and device buffers alive until the cyclic GC runs
        self._ctx = weakref.ref(ctx)
        self.lib = ctx.lib
        self.nbytes = int(nbytes)
        self.ptr = ctx.lib.frs_host_malloc(ctx.handle, self.nbytes)
        if not self.ptr:
            raise FrsError(-2, ctx.last_error())  # FRS_E_HIP
        self.array = np.frombuffer((ctypes.c_uint8 * self.nbytes).from_address(self.ptr), dtype=np.uint8)

    @property
    def ctx(self):
        return self._ctx()

    def close(self):
        if self.ptr:
            self.array = None
            c = self._ctx()
            # a buffer that outlived its context is freed without one (frs_host_free accepts a null context)
            self.lib.frs_host_free(c.handle if c is not None and c.handle else None, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One frs_ctx (one device, one HIP stream).  Not shared between threads."""

    def __init__(self, device: int = 0, lib_path: Optional[os.PathLike] = None):
        self.lib = load_library(lib_path)
        if self.lib.frs_device_count() <= 0:
            raise NativeUnavailable("no gfx950 (MI355X) device visible to HIP")
        h = ctypes.c_void_p()
        rc = self.lib.frs_ctx_create(device, ctypes.byref(h))
        if rc != FRS_OK:
            raise NativeUnavailable(f"frs_ctx_create({device}) failed: {STATUS.get(rc, rc)}")
        self.handle = h
        self.device = device
        self._pin, self._pin_view = None, None  # reusable page-locked buffer, weakref to its last exported view

    def close(self):
        if getattr(self, "handle", None):
            self.release_pinned()
            self.lib.frs_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        m = self.lib.frs_last_error(self.handle)
        return m.decode() if m else ""

    def _check(self, rc: int):
        if rc != FRS_OK:
            raise FrsError(rc, self.last_error())

    # ---- memory
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def host_buffer(self, nbytes: int) -> HostBuffer:
        return HostBuffer(self, nbytes)

    def sync(self):
        self._check(self.lib.frs_ctx_sync(self.handle))

    def pinned(self, nbytes: int) -> np.ndarray:
        """uint8[nbytes] view of a page-locked host buffer (frs_host_malloc): the arena of a large host encode lands in
        it at DMA rate.  The returned array owns the buffer (it is freed when the last view of it dies), so a view
        handed out earlier is never invalidated.  The context keeps one buffer for reuse and hands it out again only
        while no earlier view of it is alive; a request it cannot serve gets a buffer of exactly its size."""
        nbytes = int(nbytes)
        hb = self._pin
        if hb is not None and (hb.nbytes < nbytes or (self._pin_view is not None and self._pin_view() is not None)):
            # too small, or still in use by an earlier result: the context lets go of it (live views keep it)
            self._pin, self._pin_view, hb = None, None, None
        if hb is None:
            hb = HostBuffer(self, nbytes)
            self._pin = hb
        view = (ctypes.c_uint8 * hb.nbytes).from_address(hb.ptr)
        view._owner = hb  # the array's base holds the buffer alive
        self._pin_view = weakref.ref(view)
        return np.frombuffer(view, dtype=np.uint8, count=nbytes)

    def release_pinned(self):
        """Drop the context's reusable page-locked buffer (views still alive keep theirs until they die)."""
        self._pin, self._pin_view = None, None

    # ---- encode
    @staticmethod
    def make_desc(height, width, dtype, *, row_stride=None, band_stride=None, band0=0, nbands=1,
                  tile_h=512, tile_w=512, sample_rate=44100, bits_per_sample=16, blocksize=4096,
                  compression_level=5, tile_begin=0, tile_end=None, norm_mode=0) -> EncodeDesc:
        d = EncodeDesc()
        d.height, d.width = int(height), int(width)
        d.row_stride = int(row_stride if row_stride is not None else width)
        d.band_stride = int(band_stride if band_stride is not None else d.row_stride * height)
        d.dtype = DTYPE_CODES[np.dtype(dtype)]
        d.band0, d.nbands = int(band0), int(nbands)
        d.tile_h, d.tile_w = int(tile_h), int(tile_w)
        d.blocksize, d.sample_rate = int(blocksize), int(sample_rate)
        d.bits_per_sample, d.compression_level = int(bits_per_sample), int(compression_level)
        d.norm_mode = int(norm_mode)
        ntiles = ((d.height + d.tile_h - 1) // d.tile_h) * ((d.width + d.tile_w - 1) // d.tile_w)
        d.tile_begin = int(tile_begin)
        d.tile_end = int(ntiles if tile_end is None else tile_end)
        return d

    def arena_bound(self, desc: EncodeDesc) -> int:
        return int(self.lib.frs_encode_arena_bound(ctypes.byref(desc)))

    def encode_tiles_host(self, raster: np.ndarray, desc: EncodeDesc, pinned: bool = False
                          ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, int]:
        """Host-pointer encode.  Returns (arena uint8, tile_off int64[n+1], tile_min, tile_max, stream_bps).
        pinned=True: the arena is a view of the context's page-locked buffer (see pinned())."""
        r = raster if _is_window_of(raster, desc) else np.ascontiguousarray(raster)
        n = desc.tile_end - desc.tile_begin
        off = np.zeros(n + 1, dtype=np.int64)
        mn = np.zeros(max(n, 1), dtype=np.float64)
        mx = np.zeros(max(n, 1), dtype=np.float64)
        bps = ctypes.c_int32()
        cap = self.arena_bound(desc)
        arena = self.pinned(cap) if pinned else np.empty(cap, dtype=np.uint8)
        self._check(self.lib.frs_encode_tiles(
            self.handle, ctypes.byref(desc), _p(r), _p(arena), cap, off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            mn.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), mx.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
            ctypes.byref(bps)))
        return arena[: off[n]], off, mn[:n], mx[:n], bps.value

    def encode_tiles_device(self, raster_ptr: int, desc: EncodeDesc, arena: DeviceBuffer):
        """Device-resident encode (bench path).  Returns (tile_off, tile_min, tile_max, stream_bps)."""
        n = desc.tile_end - desc.tile_begin
        off = np.zeros(n + 1, dtype=np.int64)
        mn = np.zeros(max(n, 1), dtype=np.float64)
        mx = np.zeros(max(n, 1), dtype=np.float64)
        bps = ctypes.c_int32()
        self._check(self.lib.frs_encode_tiles_device(
            self.handle, ctypes.byref(desc), ctypes.c_void_p(raster_ptr), ctypes.c_void_p(arena.ptr), arena.nbytes,
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), mn.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
            mx.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(bps)))
        return off, mn[:n], mx[:n], bps.value

    # ---- decode
    def decode_frames_host(self, blob: bytes, stream_off: Sequence[int], pcm_counts: Sequence[int], channels: int,
                           bps: int, blocksize: int = 4096) -> np.ndarray:
        """Decode streams (frames only) -> int32 [sum(pcm_counts), channels]."""
        b = np.frombuffer(blob, dtype=np.uint8) if not isinstance(blob, np.ndarray) else blob
        b = np.ascontiguousarray(b)
        soff = np.ascontiguousarray(np.asarray(stream_off, dtype=np.int64))
        poff = np.zeros(len(pcm_counts) + 1, dtype=np.int64)
        poff[1:] = np.cumsum(np.asarray(pcm_counts, dtype=np.int64))
        out = np.empty((int(poff[-1]), channels), dtype=np.int32)
        self._check(self.lib.frs_decode_frames(
            self.handle, _p(b), soff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(pcm_counts), channels, bps,
            blocksize, _p(out), poff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return out

    def decode_frames_device(self, blob: DeviceBuffer, stream_off: np.ndarray, pcm_counts: Sequence[int],
                             channels: int, bps: int, pcm: DeviceBuffer, blocksize: int = 4096) -> np.ndarray:
        soff = np.ascontiguousarray(np.asarray(stream_off, dtype=np.int64))
        poff = np.zeros(len(pcm_counts) + 1, dtype=np.int64)
        poff[1:] = np.cumsum(np.asarray(pcm_counts, dtype=np.int64))
        self._check(self.lib.frs_decode_frames_device(
            self.handle, ctypes.c_void_p(blob.ptr), soff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            len(pcm_counts), channels, bps, blocksize, ctypes.c_void_p(pcm.ptr),
            poff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return poff

    def decode_tiles_host(self, blob, stream_off: Sequence[int], pcm_counts: Sequence[int], channels: int, bps: int,
                          data_min: Sequence[float], data_max: Sequence[float], dtype,
                          blocksize: int = 4096) -> np.ndarray:
        """Decode + de-normalise streams in one pass -> `dtype` [sum(pcm_counts), channels] (converter.py:241-282)."""
        b = np.frombuffer(blob, dtype=np.uint8) if not isinstance(blob, np.ndarray) else blob
        b = np.ascontiguousarray(b)
        soff = np.ascontiguousarray(np.asarray(stream_off, dtype=np.int64))
        poff = np.zeros(len(pcm_counts) + 1, dtype=np.int64)
        poff[1:] = np.cumsum(np.asarray(pcm_counts, dtype=np.int64))
        mn = np.ascontiguousarray(np.asarray(data_min, dtype=np.float64))
        mx = np.ascontiguousarray(np.asarray(data_max, dtype=np.float64))
        if len(mn) != len(pcm_counts) or len(mx) != len(pcm_counts) or len(soff) != len(pcm_counts) + 1:
            raise ValueError("one stream offset pair and one data_min/data_max per stream")
        out = np.empty((int(poff[-1]), channels), dtype=dtype)
        dp = ctypes.POINTER(ctypes.c_double)
        self._check(self.lib.frs_decode_tiles(
            self.handle, _p(b), soff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(pcm_counts), channels, bps,
            blocksize, poff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), mn.ctypes.data_as(dp),
            mx.ctypes.data_as(dp), DTYPE_CODES[np.dtype(dtype)], _p(out)))
        return out

    def decode_tiles_device(self, blob: DeviceBuffer, stream_off: np.ndarray, pcm_counts: Sequence[int], channels: int,
                            bps: int, data_min: Sequence[float], data_max: Sequence[float], dtype, out,
                            blocksize: int = 4096, blob_ptr: Optional[int] = None) -> np.ndarray:
        """Device-resident fused decode into `out` (a DeviceBuffer, or a HostBuffer the kernels store straight into);
        returns the sample offsets (pcm_off)."""
        soff = np.ascontiguousarray(np.asarray(stream_off, dtype=np.int64))
        poff = np.zeros(len(pcm_counts) + 1, dtype=np.int64)
        poff[1:] = np.cumsum(np.asarray(pcm_counts, dtype=np.int64))
        mn = np.ascontiguousarray(np.asarray(data_min, dtype=np.float64))
        mx = np.ascontiguousarray(np.asarray(data_max, dtype=np.float64))
        if int(poff[-1]) * channels * np.dtype(dtype).itemsize > out.nbytes:
            raise ValueError("output buffer too small")
        dp = ctypes.POINTER(ctypes.c_double)
        self._check(self.lib.frs_decode_tiles_device(
            self.handle, ctypes.c_void_p(blob.ptr if blob_ptr is None else blob_ptr),
            soff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(pcm_counts), channels, bps, blocksize,
            poff.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), mn.ctypes.data_as(dp), mx.ctypes.data_as(dp),
            DTYPE_CODES[np.dtype(dtype)], ctypes.c_void_p(out.ptr)))
        return poff

    def decode_tile_device(self, blob, start: int, end: int, count: int, channels: int, bps: int, data_min: float,
                           data_max: float, dtype, out, blocksize: int = 4096) -> None:
        """decode_tiles_device for ONE stream (blob bytes [start, end), `count` samples per channel) -- the latency
        path of a bbox query: argument tables are this context's reused ctypes arrays (no numpy per call)."""
        dt = _DT_CACHE.get(dtype)
        if dt is None:
            dt = _DT_CACHE[dtype] = (np.dtype(dtype).itemsize, DTYPE_CODES[np.dtype(dtype)])
        if count * channels * dt[0] > out.nbytes:
            raise ValueError("output buffer too small")
        rc = self.lib.frs_decode_tile_device(self.handle, blob.ptr, int(start), int(end), int(count), channels, bps,
                                             blocksize, float(data_min), float(data_max), dt[1], out.ptr)
        if rc != FRS_OK:
            raise FrsError(rc, self.last_error())

    def denormalize_host(self, pcm: np.ndarray, data_min: float, data_max: float, dtype, pcm_bps: int = 16) -> np.ndarray:
        p = np.ascontiguousarray(pcm, dtype=np.int32)
        out = np.empty(p.shape, dtype=dtype)
        self._check(self.lib.frs_denormalize(self.handle, _p(p), p.size, int(pcm_bps), float(data_min), float(data_max),
                                             DTYPE_CODES[np.dtype(dtype)], _p(out)))
        return out

    def denormalize_device(self, pcm_ptr: int, n: int, data_min: float, data_max: float, dtype, out_ptr: int,
                           pcm_bps: int = 16):
        self._check(self.lib.frs_denormalize_device(self.handle, ctypes.c_void_p(pcm_ptr), int(n), int(pcm_bps),
                                                    float(data_min), float(data_max), DTYPE_CODES[np.dtype(dtype)],
                                                    ctypes.c_void_p(out_ptr)))

    # ---- bench helpers
    def synth_raster(self, buf: DeviceBuffer, bands: int, height: int, width: int, row0: int = 0,
                     full_height: Optional[int] = None, seed: int = 1234):
        self._check(self.lib.frs_synth_raster_device(self.handle, ctypes.c_void_p(buf.ptr), bands, height, width, row0,
                                                     full_height if full_height is not None else height, seed))

    def profile(self, on: bool = True):
        self._check(self.lib.frs_profile_enable(self.handle, 1 if on else 0))

    def profile_avg_ms(self, kernel: str) -> float:
        return float(self.lib.frs_profile_avg_ms(self.handle, kernel.encode()))

    def profile_reset(self):
        self.lib.frs_profile_reset(self.handle)


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    """Process-wide context on device 0 (or $FRS_DEVICE / LOCAL_RANK)."""
    global _default_ctx
    if _default_ctx is None:
        dev = int(os.environ.get("FRS_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        _default_ctx = Context(dev)
    return _default_ctx
