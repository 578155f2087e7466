"""CPU checks of the oracle's two-channel (mid/side) restatement: the stereo test rasters reach all four channel
assignments and every stream decodes back to its samples.  (Parity unpinned: no reference fixture has 2 channels.)"""
import numpy as np

from oracle import oracle as O
from tests.test_gpu_stereo import _cases


def test_oracle_covers_every_assignment():
    seen = set()
    wide_side = False
    for name, arr, bits in _cases():
        B, H, W = arr.shape
        pcm, mn, mx, bps = O.normalize(arr.transpose(1, 2, 0).reshape(-1, B))
        fr = O.encode_frames(pcm, bps, 44100)
        ca = O.frame_assignments(fr, 2, bps, pcm.shape[0])
        seen |= set(int(c) for c in ca)
        assert np.array_equal(O.decode_frames(fr, 2, bps, pcm.shape[0]), pcm), name
        side = pcm[:, 0].astype(np.int64) - pcm[:, 1]
        wide_side |= bool(np.abs(side).max() >= 2 ** 31) and bool((ca == 10).any())
    assert seen == {1, 8, 9, 10}, seen
    assert wide_side  # a 33-bit side signal is written (mid-side) somewhere in the set
