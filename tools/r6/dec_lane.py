#!/usr/bin/env python3
"""Round 6 lane-decoder occupancy variants (variants/lib<name>.so, FRS_LIB_PATH):
dw4 = the tree's lane decoder (7 staged groups + the line's last from registers) in 4-wave work-groups (3 per CU);
the tree launches one-wave work-groups."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import build_variant  # noqa: E402


def wgw4(src):
    a = "#define FRS_LANE(K) k_decode_frames_lane<K, false, 1><<<(unsigned)((frames + 63) / 64), 64, lane_lds, st>>>("
    assert src.count(a) == 1
    return src.replace(a, "#define FRS_LANE(K) k_decode_frames_lane<K, false, 4><<<(unsigned)((frames + 255) / 256), 256, lane_lds, st>>>(")


if __name__ == "__main__":
    print(build_variant("dw4", wgw4, src_name="frs_decode.hip"))
