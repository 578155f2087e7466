"""Compression levels 0..5 (cli.py:36-37 `-c`, converter.py:112/204, spatial_encoder.py:137/281) in the oracle.

libFLAC's level table (docs/sonos-pyflac.txt:6926-6931) differs between levels 0..5 only in do/loose mid-side stereo,
max_lpc_order (0, 0, 0, 6, 8, 8) and max_residual_partition_order (3, 3, 3, 4, 4, 5); the window stays tukey(0.5)
and the blocksize 4096 (converter.py:205).  Parity for levels other than 5 is UNPINNED: no fixture of the reference
holds one; these tests check the restatement's structure (predictor and partition limits, lossless decode) and that
level 5 is the pinned encoder unchanged.  Levels 6..8 (subdivide_tukey) and loose mid/side (1, 4 on two channels)
are rejected by the oracle, the C-ABI and the host (converter.check_level).
"""
import numpy as np
import pytest

from flac_raster_amd.converter import check_level
from oracle import oracle as O

LIMITS = {0: (0, 3), 1: (0, 3), 2: (0, 3), 3: (6, 4), 4: (8, 4), 5: (8, 5)}  # (max lpc order, max partition order)


def level_signal(n, ch, seed, amp=3000.0):
    """Smooth signal with noise whose amplitude changes every 128 samples (high partition orders win) and a
    flat stretch (CONSTANT / low-order subframes)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    cols = []
    for c in range(ch):
        env = np.repeat(rng.choice([1.0, 4.0, 40.0, 300.0], size=n // 128 + 1), 128)[:n]
        x = amp * np.sin(t / (150.0 + 40 * c)) + 400 * np.sin(t / 9.0) * (c % 2) + env * rng.standard_normal(n)
        x[n // 3:n // 3 + 5000] = 17
        cols.append(x)
    return np.clip(np.stack(cols, axis=1), -32768, 32767).astype(np.int32)


def _ok_levels(ch):
    return [lv for lv in range(6) if not (ch == 2 and lv in (1, 4))]


@pytest.mark.parametrize("ch", [1, 2, 3])
def test_levels_lossless_and_limits(ch):
    x = level_signal(3 * 4096 + 1234, ch, 10 + ch)
    for lv in _ok_levels(ch):
        fr = O.encode_frames(x, 16, 44100, level=lv)
        assert np.array_equal(O.decode_frames(fr, ch, 16, len(x)), x), lv
        sf = O.subframe_types(fr, ch, 16, len(x))
        t, po = sf[:, 0], sf[:, 1]
        max_lpc, max_po = LIMITS[lv]
        lpc = t >= 32
        if max_lpc == 0:
            assert not lpc.any(), lv
        else:
            assert (t[lpc] - 31 <= max_lpc).all(), lv
        assert (po <= max_po).all(), lv
        if ch == 1 and lv == 5:
            assert (po == 5).any()  # the test signal reaches level 5's partition limit


def test_level5_is_default_and_mono_levels_0_to_2_agree():
    x = level_signal(5 * 4096, 1, 3)
    assert O.encode_frames(x, 16, 44100) == O.encode_frames(x, 16, 44100, level=5)
    # mono: levels 0, 1, 2 differ only in mid/side stereo
    assert O.encode_frames(x, 16, 44100, level=0) == O.encode_frames(x, 16, 44100, level=1) \
        == O.encode_frames(x, 16, 44100, level=2)
    assert O.encode_frames(x, 16, 44100, level=3) != O.encode_frames(x, 16, 44100, level=5)


def test_stereo_assignments_by_level():
    """Two channels: levels 0 and 3 code channels independently (assignment 1); levels 2 and 5 search mid/side."""
    n = 8 * 4096
    t = np.arange(n)
    rng = np.random.default_rng(5)
    L = 2000 * np.sin(t / 300.0) + rng.normal(0, 20, n)
    R = L + rng.normal(0, 3, n)  # right ~ left: side coding wins
    x = np.stack([L, R], axis=1).astype(np.int32)
    for lv in (0, 3):
        assert (O.frame_assignments(O.encode_frames(x, 16, 44100, level=lv), 2, 16, n) == 1).all(), lv
    for lv in (2, 5):
        assert (O.frame_assignments(O.encode_frames(x, 16, 44100, level=lv), 2, 16, n) >= 8).any(), lv


def test_unsupported_levels_rejected():
    x = level_signal(4096, 2, 1)
    for lv in (1, 4, 6, 8):
        with pytest.raises(ValueError):
            O.encode_frames(x, 16, 44100, level=lv)
    with pytest.raises(ValueError):
        O.encode_frames(x[:, :1], 16, 44100, level=6)
    check_level(0, 2)
    check_level(4, 1)
    check_level(5, 2)
    for lv, ch in ((1, 2), (4, 2), (6, 1), (7, 3), (8, 1)):
        with pytest.raises(NotImplementedError):
            check_level(lv, ch)
    for lv in (-1, 9):
        with pytest.raises(ValueError):
            check_level(lv, 1)
