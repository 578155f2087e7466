"""One fast-path encode with FRS_FUSED=1 on the test_fast_path_matches_oracle[int16-900-1800] band, checked against
the oracle (debugging k_fused_v6)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from flac_raster_amd import _native
from oracle import oracle as O
from tests.test_gpu_encode_parity import _gpu_tiles

H, W, tile, lo, hi = 1024, 1536, 512, 900, 1800
rng = np.random.default_rng(hash((lo, hi)) % 1000)
y, x = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
band = np.clip(lo + (hi - lo) * (0.5 + 0.45 * np.sin(6 * x) * np.cos(4 * y)) + rng.normal(0, 9.3, (H, W)), lo, hi)
band = band.astype(np.int16)
ctx = _native.Context(0)
t = time.time()
arena, off, mn, mx, bps = _gpu_tiles(ctx, band, tile)
print("gpu", time.time() - t, flush=True)
o_arena, o_off, o_mn, o_mx = O.encode_tiles(band, tile)
print("equal", arena.tobytes() == o_arena.tobytes(), list(off) == list(o_off), flush=True)
