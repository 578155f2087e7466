"""C5's early completion with the output in page-locked host memory (frs_decode_tile_device into a HostBuffer).

The optimistic pipe decode returns when the last work-group has published its completion word, before the stream's
own completion signal.  CONSTANT and VERBATIM frames are stored by the producer wave (not the consumer that exits),
so their stores must be released before that word.  Each tile here is made only of CONSTANT
frames or only of VERBATIM frames and is compared straight after the call returns, many times, with the host buffer
poisoned before each call.  A device-memory output takes the synchronising return.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

T = 512


def _tiles():
    rng = np.random.default_rng(2024)
    # CONSTANT: each 4096-sample frame (8 rows of a 512-wide tile) holds one value, values differ between frames
    const = np.repeat(rng.integers(-3000, 3000, size=T // 8, dtype=np.int16), 8 * T).reshape(T, T)
    # VERBATIM: uniform noise (no predictor beats the 16-bit samples once normalised to the full int16 range).
    # Range 16000, not the full int16 range: a tile spanning [-32768, 32766] hits the reference's NEP 50 wrap of
    # max - min (converter.py:56-86) and does not round-trip, so the equality with the band below would not hold.
    verb = rng.integers(-8000, 8000, size=(T, T), dtype=np.int16)
    return {"constant": const, "verbatim": verb}


@pytest.mark.parametrize("kind", ["constant", "verbatim"])
def test_producer_stored_frames_complete_on_return(gpu_ctx, kind):
    band = _tiles()[kind]
    d = gpu_ctx.make_desc(T, T, np.int16, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena, off, mn, mx, _ = gpu_ctx.encode_tiles_host(band, d)
    frames = np.ascontiguousarray(arena[:off[-1]])
    pcm = O.decode_frames(frames.tobytes(), 1, 16, T * T)
    ref = O.denormalize_i16(pcm, mn[0], mx[0], np.int16).reshape(-1)
    assert np.array_equal(ref, band.reshape(-1))
    # every frame is of the intended subframe type (0 CONSTANT, 1 VERBATIM): the producer wave stores them all
    types = O.subframe_types(frames.tobytes(), 1, 16, T * T)[:, 0]
    assert len(types) == T * T // 4096 and set(types.tolist()) == {0 if kind == "constant" else 1}, types
    blob = gpu_ctx.alloc(len(frames))
    blob.upload(frames)
    hb = gpu_ctx.host_buffer(T * T * 2)
    host = hb.array.view(np.int16)
    for rep in range(50):
        host[:] = -12345 if rep % 2 else 0x5A5A
        gpu_ctx.decode_tile_device(blob, 0, len(frames), T * T, 1, 16, mn[0], mx[0], np.int16, hb)
        assert np.array_equal(host, ref), (kind, rep, int(np.sum(host != ref)))
    # the same query into device memory (synchronising return), then a call after the early return
    out = gpu_ctx.alloc(T * T * 2)
    gpu_ctx.decode_tile_device(blob, 0, len(frames), T * T, 1, 16, mn[0], mx[0], np.int16, out)
    got = np.empty(T * T, dtype=np.int16)
    out.download(T * T * 2, 0, out=got.view(np.uint8))
    assert np.array_equal(got, ref)
    out.close()
    hb.close()
    blob.close()
