"""The one-launch analysis + encode (k_fused_v6) against the two-launch form and the oracle.

k_fused_v6 takes 16-bit mono jobs without partial frames (the create-streaming band-1 path, cli.py:690-763, with
libFLAC level 5 per tile): every work-group analyses tiles first and then joins the encoder, the tiles' parameters,
LUTs and frame analyses handed over between work-groups through per-tile epoch flags.  These cases cover what the
hand-off must carry: LUT tiles, constant tiles (zero normaliser), fast-division and exact-division tiles (slow
class: the sums with the fp64 normaliser inside the fused kernel), 8-frame edge tiles and 1-frame corners (frame
analyses of several tiles per 128-B line in the plain layout), a job smaller than the grid (encoders polling before
any tile is published), and repeated calls on one context (the launch epoch)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# hybrid: k_analyze_v3 takes the first 3 tiles, the fused launch the rest (both hand-off sources in one job)
FORMS = {"two_launch": {"FRS_FUSED": "0"}, "fused": {"FRS_FUSED": "1"},
         "hybrid": {"FRS_FUSED": "2", "FRS_FUSED_K": "3"}}


def _ctx(form, monkeypatch):
    from flac_raster_amd import _native
    for k, v in FORMS[form].items():
        monkeypatch.setenv(k, v)
    return _native.Context(0)


def _encode(ctx, band, tile):
    H, W = band.shape
    d = ctx.make_desc(H, W, band.dtype, tile_h=tile, tile_w=tile, sample_rate=44100, bits_per_sample=16)
    return ctx.encode_tiles_host(band, d)


def _dem(H, W, seed, lo=700, amp=300):
    rng = np.random.default_rng(seed)
    y, x = np.meshgrid(np.linspace(0, 20, H), np.linspace(0, 20, W), indexing="ij")
    return (lo + amp * np.sin(x * 0.8) * np.cos(y * 0.3) + 50 * rng.random((H, W))).astype(np.int16)


def _cases():
    rng = np.random.default_rng(5)
    small = _dem(1024, 1536, 1)                       # 6 tiles, 96 work-groups: most encoders poll at once
    small[:256, :256] = small[0, 0]
    edges = _dem(1088, 1600, 2)                       # 512-px tiles + 64-px edge tiles (8 frames) + 64x64 corner
    edges[512:1024, 512:1024] = 1234                  # a constant tile (zero normaliser)
    wide = rng.integers(0, 40000, size=(1024, 1024)).astype(np.uint16)   # fast reciprocal division
    wrap = rng.integers(-30000, 30000, size=(512, 1024)).astype(np.int16)  # wrapping int16: exact division
    return {"small": (small, 512), "edges": (edges, 512), "fastdiv": (wide, 512), "slow": (wrap, 512),
            "tiles64": (_dem(512, 2048, 3), 64)}


CASES = _cases()


@pytest.mark.parametrize("case", list(CASES))
def test_fused_matches_two_launch_and_oracle(case, monkeypatch):
    band, tile = CASES[case]
    outs = {}
    for form in FORMS:
        ctx = _ctx(form, monkeypatch)
        try:
            outs[form] = _encode(ctx, band, tile)
        finally:
            ctx.close()
    o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile, threads=8)
    for form, (arena, off, mn, mx, bps) in outs.items():
        assert list(off) == list(o_off), form
        assert arena.tobytes() == o_arena.tobytes(), form
        assert list(mn) == list(o_mn) and list(mx) == list(o_mx), form


@pytest.mark.parametrize("form", ["fused", "hybrid"])
def test_fused_repeated_calls_and_regrown_buffers(form, monkeypatch):
    """Launch epochs: many calls on one context, jobs growing and shrinking (new flag allocations), each byte-equal
    to the oracle."""
    ctx = _ctx(form, monkeypatch)
    try:
        for i, (H, W) in enumerate([(512, 512), (1024, 1536), (512, 512), (2048, 2048), (1024, 512), (512, 512)]):
            band = _dem(H, W, 10 + i)
            arena, off, mn, mx, bps = _encode(ctx, band, 512)
            o_arena, o_off, _, _ = O.encode_tiles(band, 512, threads=8)
            assert list(off) == list(o_off) and arena.tobytes() == o_arena.tobytes(), (H, W)
    finally:
        ctx.close()
