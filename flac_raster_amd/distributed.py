"""Multi-GPU create-streaming: tiles shard by contiguous tile rows, one process per GPU.

SURVEY 8(e): the only exchange is an all-gather of per-tile compressed sizes (int64, a few KB).  On MI355X it
is RCCL over xGMI through the codec library's C-ABI (frs_comm_*, librccl.so loaded at run time): no PyTorch.
Every rank then knows every tile's byte offset, builds the identical JSON index locally, and writes its own
tiles into the shared output file with pwritev at 4 + len(index) + byte_offset; rank 0 also writes the index
header and sets the file size.  No tile data crosses GPUs.

Ranks find each other through the usual launcher environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR,
MASTER_PORT -- torchrun's or flac_raster_amd.launch's).  Rank 0's ncclUniqueId reaches the other ranks through
a host bootstrap (TcpComm: a star of TCP connections to rank 0 on MASTER_PORT + 1 unless FRS_COMM_PORT is set);
TcpComm is also the exchange of the CPU-only tests.
"""
from __future__ import annotations

import ctypes
import os
import socket
import struct
import time
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import container, geotiff
from .streaming import EncodedTiles, streaming_headers, streaming_head, tile_grid, write_tiles


def shard_tile_rows(n_tile_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced tile-row range [tr0, tr1) of `rank` (C4: 79 rows over 8 -> 9/10 each)."""
    return rank * n_tile_rows // world, (rank + 1) * n_tile_rows // world


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    return rank, world, int(os.environ.get("LOCAL_RANK", str(rank)))


# ------------------------------------------------------------------------------------------------ host exchange
def _send_frame(s: socket.socket, b: bytes):
    s.sendall(struct.pack("<Q", len(b)) + b)


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        c = s.recv(n - len(buf))
        if not c:
            raise ConnectionError("peer closed the bootstrap connection")
        buf += c
    return bytes(buf)


def _recv_frame(s: socket.socket) -> bytes:
    return _recv_exact(s, struct.unpack("<Q", _recv_exact(s, 8))[0])


class TcpComm:
    """All-gather of byte strings over a TCP star (rank 0 is the hub).  Bootstrap of RcclComm and the exchange of
    the CPU tests; each call is one round trip per rank."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29600,
                 timeout: Optional[float] = None):
        # a dead peer closes its socket (EOF -> ConnectionError at once); a hung one is cut off after `timeout`
        # seconds of silence ($FRS_COMM_TIMEOUT, default 120 s)
        timeout = float(os.environ.get("FRS_COMM_TIMEOUT", "120")) if timeout is None else timeout
        self.rank, self.world = rank, world
        self.peers: List[socket.socket] = []
        self.sock: Optional[socket.socket] = None
        if world == 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(timeout)
            peers = {}
            while len(peers) < world - 1:
                c, _ = srv.accept()
                c.settimeout(timeout)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                r = struct.unpack("<i", _recv_exact(c, 4))[0]
                peers[r] = c
            srv.close()
            self.peers = [peers[r] for r in range(1, world)]
        else:
            t_end = time.time() + timeout
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=timeout)
                    break
                except OSError:
                    if time.time() > t_end:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", rank))
            self.sock = s

    def allgather_bytes(self, b: bytes) -> List[bytes]:
        if self.world == 1:
            return [b]
        if self.rank == 0:
            parts = [b] + [_recv_frame(p) for p in self.peers]
            blob = b"".join(struct.pack("<Q", len(x)) for x in parts) + b"".join(parts)
            for p in self.peers:
                _send_frame(p, blob)
        else:
            _send_frame(self.sock, b)
            blob = _recv_frame(self.sock)
        lens = struct.unpack(f"<{self.world}Q", blob[:8 * self.world])
        out, pos = [], 8 * self.world
        for n in lens:
            out.append(blob[pos:pos + n])
            pos += n
        return out

    def allgather_i64(self, local: np.ndarray) -> np.ndarray:
        """Equal-length int64 vectors -> concatenation in rank order."""
        parts = self.allgather_bytes(np.ascontiguousarray(local, dtype="<i8").tobytes())
        return np.frombuffer(b"".join(parts), dtype="<i8").astype(np.int64)

    def barrier(self):
        self.allgather_bytes(b"")

    def close(self):
        for p in self.peers:
            p.close()
        if self.sock:
            self.sock.close()
        self.peers, self.sock = [], None


class RcclComm:
    """RCCL communicator of the codec library (frs_comm_*): all-gather over xGMI on the context's stream."""

    def __init__(self, ctx, rank: int, world: int, boot: TcpComm):
        self.ctx, self.rank, self.world = ctx, rank, world
        L = ctx.lib
        self._L = L
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            ctx._check(L.frs_comm_unique_id(uid))
        ids = boot.allgather_bytes(bytes(uid))
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(ids[0])
        h = ctypes.c_void_p()
        ctx._check(L.frs_comm_init(ctx.handle, uid, world, rank, ctypes.byref(h)))
        self.handle = h
        self.boot = boot

    def allgather_i64(self, local: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(local, dtype=np.int64)
        out = np.empty(a.size * self.world, dtype=np.int64)
        p64 = ctypes.POINTER(ctypes.c_int64)
        self.ctx._check(self._L.frs_comm_allgather_i64(self.handle, a.ctypes.data_as(p64), a.size,
                                                       out.ctypes.data_as(p64)))
        return out

    def barrier(self):
        self.allgather_i64(np.zeros(1, dtype=np.int64))

    def close(self):
        if getattr(self, "handle", None):
            self._L.frs_comm_destroy(self.handle)
            self.handle = None
        self.boot.close()


def init_comm(ctx=None, backend: str = "rccl", rank: Optional[int] = None, world: Optional[int] = None):
    """Communicator for this rank from the launcher environment: "rccl" (GPU, needs ctx) or "tcp" (host only)."""
    r, w, _ = env_rank_world()
    rank = r if rank is None else rank
    world = w if world is None else world
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("FRS_COMM_PORT", str(int(os.environ.get("MASTER_PORT", "29500")) + 1)))
    boot = TcpComm(rank, world, addr, port)
    if backend == "tcp":
        return boot
    return RcclComm(ctx, rank, world, boot)


# ----------------------------------------------------------------------------------------- sharded create-streaming
def all_gather_sizes(local: np.ndarray, counts: Sequence[int], comm) -> np.ndarray:
    """All-gather variable-length int64 vectors (padded to the max count) -> concatenation in rank order."""
    m = max(counts)
    buf = np.zeros(m, dtype=np.int64)
    buf[:len(local)] = local
    g = comm.allgather_i64(buf).reshape(len(counts), m)
    return np.concatenate([g[r, :c] for r, c in enumerate(counts)])


def create_streaming_sharded(band_rows: np.ndarray, row0: int, full_shape: Tuple[int, int], transform, crs: Optional[str],
                             tile: int, output: Path, comm, encode: Callable[[np.ndarray, int], EncodedTiles],
                             timings: Optional[dict] = None) -> dict:
    """Rank-local part of a distributed create-streaming (cli.py:620-804 split over the ranks).

    band_rows: this rank's slab of band 1 (rows [row0, row0 + h)), starting on a tile-row boundary.
    encode:    (slab, tile) -> EncodedTiles for the slab's tiles (the GPU codec in production).
    The file is complete when every rank has returned (a final barrier).
    """
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    H, W = full_shape
    rank, world = comm.rank, comm.world
    tcols = (W + tile - 1) // tile
    trows = (H + tile - 1) // tile
    counts = [(shard_tile_rows(trows, world, r)[1] - shard_tile_rows(trows, world, r)[0]) * tcols for r in range(world)]
    if band_rows.shape[0] and row0 % tile:
        raise ValueError("a rank's slab must start on a tile-row boundary")
    if band_rows.shape[0] == 0 or band_rows.shape[1] == 0:
        # more ranks than tile rows: nothing to encode, but the rank still joins the all-gather and the barrier
        z = np.zeros(0, dtype=np.float64)
        enc = EncodedTiles([], np.zeros(0, dtype=np.uint8), np.zeros(1, dtype=np.int64), z, z, 16)
    else:
        enc = encode(band_rows, tile)
    t1 = time.perf_counter()
    all_windows = tile_grid(H, W, tile)
    first = sum(counts[:rank])
    mine = all_windows[first:first + counts[rank]]
    headers, _, _ = streaming_headers(enc, transform, crs, W, H, tile, band_rows.dtype, windows=mine)
    local = np.array([len(h) for h in headers], dtype=np.int64) + np.diff(enc.tile_off)
    sizes = all_gather_sizes(local, counts, comm)  # the one collective of the data path
    t2 = time.perf_counter()
    offs = np.zeros(len(sizes) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(sizes)
    index = {"crs": str(crs), "transform": list(transform), "width": W, "height": H, "tile_size": tile, "frames": []}
    for i, (col, row, w, h) in enumerate(all_windows):
        tt = geotiff.window_transform(transform, col, row)
        xmin, ymax = tt.c, tt.f
        index["frames"].append({"frame_id": i, "bbox": [xmin, ymax + (h * tt.e), xmin + (w * tt.a), ymax],
                                "window": {"col_off": col, "row_off": row, "width": w, "height": h},
                                "byte_offset": int(offs[i]), "byte_size": int(sizes[i])})
    head = streaming_head(index)
    fd = os.open(output, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        if rank == 0:  # safe at any time: every rank writes inside [0, total)
            os.ftruncate(fd, len(head) + int(offs[-1]))
            os.pwrite(fd, head, 0)
        write_tiles(fd, len(head) + int(offs[first]), headers, enc)
    finally:
        os.close(fd)
    comm.barrier()
    t3 = time.perf_counter()
    tm.update(encode_s=t1 - t0, exchange_s=t2 - t1, write_s=t3 - t2, total_s=t3 - t0)
    return index


def gpu_encoder(ctx):
    """The production `encode` of create_streaming_sharded: the rank's GPU codec."""
    from .streaming import encode_band_tiles
    return lambda slab, tile: encode_band_tiles(slab, tile, ctx)


def create_streaming_distributed(input_file: Path, output_file: Path, tile_size: int = 1024,
                                 backend: Optional[str] = None) -> dict:
    """One rank of `create-streaming` over the launcher's ranks: reads the GeoTIFF, encodes its tile rows on GPU
    LOCAL_RANK, all-gathers the tile sizes and writes its tiles into the shared output file.  backend: "rccl"
    (default) or "tcp" ($FRS_COMM_BACKEND; the host exchange, e.g. for ranks sharing one GPU in tests)."""
    from ._native import Context, device_count
    backend = backend or os.environ.get("FRS_COMM_BACKEND", "rccl")
    rank, world, local_rank = env_rank_world()
    with geotiff.TiffFile(input_file) as tf:  # only this rank's band-1 rows are decoded (cli.py:698-699)
        H, W = tf.height, tf.width
        tr0, tr1 = shard_tile_rows((H + tile_size - 1) // tile_size, world, rank)
        transform, epsg, _, _ = tf.georef()
        slab = np.ascontiguousarray(tf.read_rows(tr0 * tile_size, min(tr1 * tile_size, H), [0])[0])
    transform = transform or geotiff.Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0)
    crs = f"EPSG:{epsg}" if epsg else None
    ndev = device_count()
    if backend == "rccl" and world > ndev:
        raise RuntimeError(f"{world} ranks but {ndev} GPUs: one rank per GPU (FRS_COMM_BACKEND=tcp shares GPUs)")
    ctx = Context(local_rank % max(1, ndev))
    comm = init_comm(ctx, backend)
    try:
        return create_streaming_sharded(slab, tr0 * tile_size, (H, W), transform, crs, tile_size,
                                        Path(output_file), comm, gpu_encoder(ctx))
    finally:
        comm.close()
        ctx.close()
