"""Compression levels 0..8 (cli.py:36-37 `-c`, converter.py:112/204, spatial_encoder.py:137/281) in the oracle.

libFLAC's level table (docs/sonos-pyflac.txt:6926-6934): do/loose mid-side stereo, max_lpc_order (0, 0, 0, 6, 8, 8,
8, 12, 12), max_residual_partition_order (3, 3, 3, 4, 4, 5, 6, 6, 6) and the apodization -- tukey(0.5) up to level 5,
subdivide_tukey(2) at 6 and 7, subdivide_tukey(3) at 8 (several windows per subframe, the best LPC candidate kept);
levels 1 and 4 on two channels use loose mid/side (a full independent-vs-mid/side evaluation every
round(0.4 s / block) frames, the previous choice in between).  Parity for levels other than 5 is UNPINNED: no fixture
of the reference holds one; these tests check the restatement's structure (predictor and partition limits, lossless
decode, the loose mid/side schedule) and that level 5 is the pinned encoder unchanged.
"""
import numpy as np
import pytest

from flac_raster_amd.converter import check_level
from oracle import oracle as O

LIMITS = {0: (0, 3), 1: (0, 3), 2: (0, 3), 3: (6, 4), 4: (8, 4), 5: (8, 5), 6: (8, 6), 7: (12, 6), 8: (12, 6)}
# (max lpc order, max partition order)


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
    return list(range(9))


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


def test_levels_6_to_8_use_their_windows_and_orders():
    """Level 7/8 reach LPC orders above 8 on a resonant signal; levels 6..8 differ from level 5 and from each other
    (extra windows / orders); every level decodes losslessly."""
    n = 6 * 4096
    t = np.arange(n)
    rng = np.random.default_rng(21)
    x = (6000 * np.sin(t / 7.3) + 5000 * np.sin(t / 3.1) + 3000 * np.sin(t / 2.05) + 2000 * np.sin(t / 1.37) +
         1500 * np.sin(t / 1.11) + 900 * np.sin(t / 0.83) + rng.normal(0, 2, n)).astype(np.int32)[:, None]
    fr = {lv: O.encode_frames(x, 16, 44100, level=lv) for lv in (5, 6, 7, 8)}
    for lv, f in fr.items():
        assert np.array_equal(O.decode_frames(f, 1, 16, n), x), lv
    o7 = O.subframe_types(fr[7], 1, 16, n)[:, 0]
    assert ((o7 >= 32) & (o7 - 31 > 8)).any()  # orders 9..12
    assert len({fr[5], fr[6], fr[7], fr[8]}) == 4
    # the best of several windows: level 8's estimate-driven choice is never larger than one window's on this signal
    assert len(fr[8]) <= len(fr[7]) * 1.01


def test_loose_mid_side_schedule():
    """Levels 1 and 4 on two channels: assignments are independent (1) or mid-side (10) only, and change only on the
    evaluation frames (every round(44100 * 0.4 / 4096) = 4 frames from frame 0)."""
    n = 24 * 4096
    t = np.arange(n)
    rng = np.random.default_rng(8)
    L = 3000 * np.sin(t / 200.0) + rng.normal(0, 30, n)
    R = np.where((t // 4096) % 6 < 3, L + rng.normal(0, 2, n), rng.normal(0, 3000, n))  # correlated, then not
    x = np.clip(np.stack([L, R], axis=1), -32768, 32767).astype(np.int32)
    for lv in (1, 4):
        f = O.encode_frames(x, 16, 44100, level=lv)
        assert np.array_equal(O.decode_frames(f, 2, 16, n), x)
        ca = O.frame_assignments(f, 2, 16, n)
        assert set(np.unique(ca)) <= {1, 10}, lv
        assert {1, 10} <= set(np.unique(ca)), lv  # both chosen somewhere
        for k in range(1, len(ca)):
            if k % 4:
                assert ca[k] == ca[k - 1], (lv, k)
    # the exhaustive search (level 5) on the same signal picks left-side (8) on some frames, which loose mid/side never
    # considers
    assert 8 in set(np.unique(O.frame_assignments(O.encode_frames(x, 16, 44100, level=5), 2, 16, n)))


def test_product_level_gate():
    """The host accepts every level the GPU kernels implement (converter.check_level)."""
    check_level(0, 2)
    check_level(4, 1)
    check_level(5, 2)
    for lv in (-1, 9):
        with pytest.raises(ValueError):
            check_level(lv, 1)
