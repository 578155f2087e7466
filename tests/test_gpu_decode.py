"""GPU decode parity: the mono 16-bit decoders (k_decode_frames_pipe: scalar-unit Rice decode + v_dot2 LPC restore
in two waves; k_decode_frames_lane: one lane per frame) and the lane-0 wave decoder must all return exactly the
oracle's decode of the same frames,
for every subframe type the encoder emits (CONSTANT, VERBATIM, FIXED, LPC, wasted bits), partial frames,
Rice windows that hit the 64-code cap and codes longer than a 64-bit candidate window."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _header_len(frames: np.ndarray) -> int:
    """Bytes of the first frame's header up to and including its CRC-8 (RFC 9639 9.1)."""
    b = frames.tobytes()
    n = 4
    v = b[n]
    n += 1 + (0 if v < 0x80 else 1 if v < 0xE0 else 2 if v < 0xF0 else 3)
    bsc, src = b[2] >> 4, b[2] & 15
    n += {6: 1, 7: 2}.get(bsc, 0) + {12: 1, 13: 2, 14: 2}.get(src, 0)
    return n + 1


def _bands():
    rng = np.random.default_rng(77)
    H, W = 512, 768
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    dem = (1000 + 300 * np.sin(x * 0.8) * np.cos(y * 0.3) + 150 * np.sin(1.2 * x) * np.sin(1.1 * y)
           + 50 * rng.random((H, W))).astype(np.int16)
    dem[:64, :128] = dem[0, 0]                                     # constant frames
    noise = rng.integers(-32768, 32767, size=(256, 256), dtype=np.int16)  # verbatim-heavy
    steps = (np.arange(320 * 200).reshape(320, 200) // 7 % 50 * 64).astype(np.uint16)  # wasted bits
    odd = (700 + 40 * np.sin(np.linspace(0, 30, 300 * 333)).reshape(300, 333)
           + rng.normal(0, 3, (300, 333))).astype(np.int16)  # partial frames, rows crossing frames
    # Rice-window edge cases of the pipelined decoder: near-flat data (Rice parameter 0-1, so a 1024-bit window
    # holds more than its 64-code cap) and a smooth field with sparse spikes (unary runs longer than 64 bits:
    # the producer's "long code" path through the scalar reader)
    flat = (100 + rng.integers(-1, 2, size=(256, 256))).astype(np.int16)
    flat[::5, :] = 100
    spiky = (500 + 20 * np.sin(np.linspace(0, 12, 256 * 256)).reshape(256, 256)).astype(np.int16)
    spiky.flat[rng.choice(spiky.size, 40, replace=False)] = rng.choice([-30000, 30000], 40).astype(np.int16)
    # uint8 output through the decoders' 8-byte vector stores (tile 200: a 3136-sample last frame)
    u8 = (128 + 90 * np.sin(np.linspace(0, 40, 400 * 600)).reshape(400, 600) + rng.normal(0, 4, (400, 600))
          ).clip(0, 255).astype(np.uint8)
    return [("dem", dem, 256), ("noise", noise, 128), ("steps", steps, 160), ("odd", odd, 128),
            ("flat", flat, 256), ("spiky", spiky, 256), ("u8", u8, 200)]


DECODERS = {"pipe": {"FRS_DECODE_LANE": "0"},      # two-wave pipelined decoder (latency; C5 queries), optimistic:
            #                                       candidates = frames, CRC-16 checked inside the decoder
            "pipe_chain": {"FRS_DECODE_LANE": "0", "FRS_PIPE_OPT": "0"},  # the same after the span check + chain
            "lane": {"FRS_DECODE_LANE": "1"},      # lane-per-frame decoder (throughput; batched decodes)
            "wave": {"FRS_FORCE_GENERIC": "1"}}    # one-lane wave decoder (any layout)


def _decoder_ctx(kind, monkeypatch):
    from flac_raster_amd import _native
    for k, v in DECODERS[kind].items():
        monkeypatch.setenv(k, v)
    return _native.Context(0)


@pytest.mark.parametrize("kind", list(DECODERS))
def test_decode_matches_oracle(gpu_ctx, kind, monkeypatch):
    dctx = _decoder_ctx(kind, monkeypatch)
    for name, band, tile in _bands():
        H, W = band.shape
        d = gpu_ctx.make_desc(H, W, band.dtype, tile_h=tile, tile_w=tile, sample_rate=44100, bits_per_sample=16)
        arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
        counts = []
        for r0 in range(0, H, tile):
            for c0 in range(0, W, tile):
                counts.append(min(tile, H - r0) * min(tile, W - c0))
        pcm = dctx.decode_frames_host(arena, off, counts, channels=1, bps=16)
        # fused decode + de-normalisation (converter.py:241-282 in one pass) against the oracle's two steps
        vals = dctx.decode_tiles_host(arena, off, counts, channels=1, bps=16, data_min=mn, data_max=mx,
                                      dtype=band.dtype)
        for t, n in enumerate(counts):
            frames = arena[off[t]:off[t + 1]].tobytes()
            ref = O.decode_frames(frames, 1, 16, n)
            a, b = int(np.sum(counts[:t])), int(np.sum(counts[:t + 1]))
            assert np.array_equal(pcm[a:b], ref), (name, t)
            assert np.array_equal(vals[a:b], O.denormalize_i16(ref, mn[t], mx[t], band.dtype)), (name, t)
    dctx.close()


@pytest.mark.parametrize("kind", list(DECODERS))
def test_decode_corrupt_streams_report_errors(gpu_ctx, kind, monkeypatch):
    """Damaged data must end in FrsError (CRC-16 span check fails, chain broken, or no sync codes at all), never a
    fault, a stall or a silent wrong decode; the context then still decodes good data (the decode path launches its
    span and frame kernels before the host knows the candidate count, so the unchained frames are skipped on
    device: a frame whose CRC span fails is never handed to a decoder)."""
    from flac_raster_amd import _native
    dctx = _decoder_ctx(kind, monkeypatch)
    band = _bands()[0][1][:256, :256].copy()
    d = gpu_ctx.make_desc(256, 256, band.dtype, tile_h=128, tile_w=128, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
    counts = [128 * 128] * 4
    flipped = arena.copy()
    flipped[off[1] + 200:off[1] + 260] ^= 0x5A  # inside tile 1's first frame
    with pytest.raises(_native.FrsError):
        dctx.decode_frames_host(flipped, off, counts, channels=1, bps=16)
    # a frame that is not the first: tile 2's third frame (the chain breaks in the middle of a stream)
    third = off[2] + (off[3] - off[2]) * 2 // 4 + 100
    flipped = arena.copy()
    flipped[third:third + 48] ^= 0xA5
    with pytest.raises(_native.FrsError):
        dctx.decode_tiles_host(flipped, off, counts, channels=1, bps=16, data_min=mn, data_max=mx, dtype=band.dtype)
    with pytest.raises(_native.FrsError):  # no sync codes anywhere
        dctx.decode_frames_host(np.zeros_like(arena), off, counts, channels=1, bps=16)
    # a crafted range where a valid frame header repeats every few bytes: more sync candidates than the bounded
    # selection keeps -> rejected before anything is written past the candidate buffer
    one = arena[:_header_len(arena)].tobytes()
    spam = np.frombuffer(one * (400000 // len(one)), dtype=np.uint8)
    with pytest.raises(_native.FrsError, match="candidates"):
        dctx.decode_frames_host(spam, [0, len(spam)], [4096 * 2], channels=1, bps=16)
    pcm = dctx.decode_frames_host(arena, off, counts, channels=1, bps=16)
    for t in range(4):
        ref = O.decode_frames(arena[off[t]:off[t + 1]].tobytes(), 1, 16, counts[t])
        assert np.array_equal(pcm[t * counts[t]:(t + 1) * counts[t]], ref), t
    dctx.close()


@pytest.mark.parametrize("kind", ["lane", "wave"])
@pytest.mark.parametrize("bands,dtype", [(3, np.uint8), (4, np.int16), (6, np.uint16)])
def test_multichannel_decode_matches_oracle(gpu_ctx, kind, bands, dtype, monkeypatch):
    """Plain-convert streams of >= 3 interleaved channels (converter.py:241-282): the lane decoder walks each frame's
    subframes into a channel-planar scratch and k_interleave_dn interleaves / de-normalises ("lane"); the one-lane
    wave decoder ("wave") is the reference layout.  Both equal the oracle's decode of the same frames, including a
    partial last frame and VERBATIM / CONSTANT subframes."""
    rng = np.random.default_rng(5 + bands)
    H, W = 300, 701
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    data = np.stack([900 + 300 * np.sin(x * (0.5 + 0.1 * b)) * np.cos(y * 0.3) + 40 * rng.random((H, W))
                     for b in range(bands)])
    if dtype == np.uint8:
        data = data / 8
    data = data.astype(dtype)
    data[1, :40, :] = data[1, 0, 0]                          # constant subframes in channel 1
    data[2, 100:140, :] = rng.integers(0, 255, size=(40, W))  # noisy (VERBATIM-leaning) rows in channel 2
    pcm_ref, mn, mx, bps = O.normalize(data.transpose(1, 2, 0).reshape(-1, bands))
    frames = np.frombuffer(O.encode_frames(pcm_ref, bps, 44100), dtype=np.uint8)
    dctx = _decoder_ctx(kind, monkeypatch)
    n = H * W
    pcm = dctx.decode_frames_host(frames, [0, frames.size], [n], channels=bands, bps=bps)
    ref = O.decode_frames(frames.tobytes(), bands, bps, n)
    assert np.array_equal(pcm.reshape(-1), ref.reshape(-1))
    vals = dctx.decode_tiles_host(frames, [0, frames.size], [n], channels=bands, bps=bps, data_min=[mn], data_max=[mx],
                                  dtype=dtype)
    assert np.array_equal(vals.reshape(-1), O.denormalize_i16(ref, mn, mx, dtype).reshape(-1))
    assert np.array_equal(vals.reshape(H, W, bands).transpose(2, 0, 1), data)  # lossless round trip
    dctx.close()


@pytest.mark.parametrize("kind", ["lane", "pipe"])
def test_long_stream_chain_matches_oracle(gpu_ctx, kind, monkeypatch):
    """One stream of more frames than k_chain_lds's LDS table (4096; a plain convert of a large raster is one stream):
    its frames are ranked in parallel (the verified sync candidates in position order, every link checked) instead of
    a dependent walk; the decode equals the oracle's, and a frame broken in the middle still ends in FrsError."""
    from flac_raster_amd import _native
    rng = np.random.default_rng(11)
    H, W = 2304, 8192
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 60, W), indexing="ij")
    band = (1000 + 300 * np.sin(x * 0.8) * np.cos(y * 0.3) + 60 * rng.random((H, W))).astype(np.int16)
    d = gpu_ctx.make_desc(H, W, band.dtype, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
    n = H * W
    assert n // 4096 > 4096
    dctx = _decoder_ctx(kind, monkeypatch)
    pcm = dctx.decode_frames_host(arena, off, [n], channels=1, bps=16)
    assert np.array_equal(pcm, O.decode_frames(arena.tobytes(), 1, 16, n))
    vals = dctx.decode_tiles_host(arena, off, [n], channels=1, bps=16, data_min=mn, data_max=mx, dtype=band.dtype)
    assert np.array_equal(vals.reshape(H, W), band)
    flipped = arena.copy()
    mid = int(off[1]) * 7 // 10
    flipped[mid:mid + 64] ^= 0x5A
    with pytest.raises(_native.FrsError):
        dctx.decode_frames_host(flipped, off, [n], channels=1, bps=16)
    dctx.close()


def test_decode_rejects_reversed_offsets(gpu_ctx):
    """Reversed stream / sample offsets are an argument error (checked before any staging is sized)."""
    from flac_raster_amd import _native
    blob = np.zeros(64, dtype=np.uint8)
    for call in (lambda: gpu_ctx.decode_tiles_host(blob, [40, 0], [4096], channels=1, bps=16, data_min=[0.0],
                                                   data_max=[1.0], dtype=np.int16),
                 lambda: gpu_ctx.decode_frames_host(blob, [40, 0], [4096], channels=1, bps=16)):
        with pytest.raises(_native.FrsError) as e:
            call()
        assert e.value.code == -1 and "non-decreasing" in str(e.value)


def _crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def _crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _wrapping_lpc_frames(nframes: int, bs: int = 64) -> bytes:
    """Hand-built mono 16-bit frames (RFC 9639) whose LPC prediction sum needs more than 32 bits: order 8, 15-bit
    coefficients of 16383, shift 14, every sample 32767 -> sum q.x = 8 * 16383 * 32767 > 2^31.  libFLAC decodes
    them with its 64-bit restore (prec + bps + log2(order) > 32); a decoder summing mod 2^32 must notice."""
    out = bytearray()
    for fno in range(nframes):
        bits = []

        def put(v, n):
            for i in range(n - 1, -1, -1):
                bits.append((v >> i) & 1)
        hdr = bytes([0xFF, 0xF8, (7 << 4) | 9, (0 << 4) | (4 << 1)])
        assert fno < 128
        hdr += bytes([fno]) + (bs - 1).to_bytes(2, "big")
        hdr += bytes([_crc8(hdr)])
        o, prec, shift, q, x = 8, 15, 14, 16383, 32767
        put(0, 1)
        put(32 + o - 1, 6)
        put(0, 1)
        for _ in range(o):
            put(x & 0xFFFF, 16)
        put(prec - 1, 4)
        put(shift, 5)
        for _ in range(o):
            put(q & 0x7FFF, 15)
        put(0, 2)   # Rice, 4-bit parameters
        put(0, 4)   # partition order 0
        k = 14
        put(k, 4)
        r = x - ((o * q * x) >> shift)
        u = (r << 1) ^ (r >> 63) if r >= 0 else ((-r) << 1) - 1
        for _ in range(bs - o):
            put(0, u >> k)
            put(1, 1)
            put(u & ((1 << k) - 1), k)
        while len(bits) % 8:
            bits.append(0)
        body = hdr + bytes(int("".join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8))
        out += body + _crc16(body).to_bytes(2, "big")
    return bytes(out)


@pytest.mark.parametrize("kind", list(DECODERS))
def test_wrapped_lpc_prediction_decodes_exactly(gpu_ctx, kind, monkeypatch):
    """The 32-bit restore paths sum the LPC prediction mod 2^32 (level 5's 16-bit precision choice reaches
    prec + bps + log2(order) = 32); a wrapped sum must be detected and the subframe redone exactly."""
    nf, bs = 80, 64  # > 64 frames: the lane decoder takes the job when forced
    fr = _wrapping_lpc_frames(nf, bs)
    n = nf * bs
    ref = O.decode_frames(fr, 1, 16, n)
    assert np.all(ref == 32767)
    dctx = _decoder_ctx(kind, monkeypatch)
    got = dctx.decode_frames_host(np.frombuffer(fr, np.uint8), [0, len(fr)], [n], channels=1, bps=16, blocksize=bs)
    assert np.array_equal(got.reshape(-1), ref.reshape(-1))
    dctx.close()


@pytest.mark.parametrize("span", ["pcrc", "read"])
def test_large_range_dense_candidates_lossless(gpu_ctx, span, monkeypatch):
    """Ranges above 16 MB take the two-pass selection: per-64-KB-block counts that keep up to 32 candidate positions
    per block, a scan, and a placement pass that copies them (a block with more candidates re-reads its bytes).
    Ramps code to tiny frames (hundreds of sync candidates per block: the re-read path), noise in the other half of
    the same job to ~8 KB frames (the kept-positions path); all tiles decode losslessly in one call.  span="pcrc": the
    span check from the prefix CRCs the selection folds (k_span_pcrc); "read": the span check that reads every frame
    again (k_span_crc_lane).  A flipped byte anywhere ends in FrsError either way."""
    from flac_raster_amd import _native, streaming
    monkeypatch.setenv("FRS_SPAN_READ", "1" if span == "read" else "2")
    rng = np.random.default_rng(5)
    H, W, T = 6144, 6144, 512
    y, x = np.mgrid[0:H, 0:W]
    # ramps: tiny FIXED frames, hundreds of syncs per block; small-range noise: ~8 KB frames (C4-like).  Ranges stay
    # small enough for the reference's normalise / de-normalise round trip to be exact (it is not for ranges near
    # 2^16, where n / 32768 against the encoder's 32767 scale moves a sample by one)
    band = ((7 * x + 3 * y) % 4000).astype(np.int16)
    band[:, W // 2:] = (1000 + rng.integers(-40, 41, size=(H, W // 2))).astype(np.int16)
    d = gpu_ctx.make_desc(H, W, band.dtype, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, bps = gpu_ctx.encode_tiles_host(band, d)
    assert off[-1] > (16 << 20)  # the two-pass selection
    counts = [w * h for (_, _, w, h) in streaming.tile_grid(H, W, T)]
    vals = gpu_ctx.decode_tiles_host(arena, off, counts, channels=1, bps=16, data_min=mn, data_max=mx,
                                     dtype=band.dtype)
    a = 0
    for (c0, r0, w, h), n in zip(streaming.tile_grid(H, W, T), counts):
        assert np.array_equal(vals[a:a + n].reshape(h, w), band[r0:r0 + h, c0:c0 + w]), (r0, c0)
        a += n
    pcm = gpu_ctx.decode_frames_host(arena, off, counts, channels=1, bps=16)
    for t in (0, len(counts) // 2 + 3, len(counts) - 1):  # a ramp tile, a noise tile, the last tile
        ref = O.decode_frames(arena[off[t]:off[t + 1]].tobytes(), 1, 16, counts[t])
        assert np.array_equal(pcm[int(np.sum(counts[:t])):int(np.sum(counts[:t + 1]))], ref), t
    for pos in (int(off[1]) + 37, int(off[len(counts) // 2 + 3]) + 5000, int(off[-1]) - 3):  # frame bodies, a footer
        flipped = arena.copy()
        flipped[pos] ^= 0x10
        with pytest.raises(_native.FrsError):
            gpu_ctx.decode_frames_host(flipped, off, counts, channels=1, bps=16)
