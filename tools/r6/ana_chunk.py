#!/usr/bin/env python3
"""Round 6 analysis chunk variants (variants/lib<name>.so, FRS_LIB_PATH): the tree's prefetching form loads 32-sample
chunks (107 VGPRs: 4 waves per SIMD, where the 64-sample prefetch needed 136 and ran at 3);
a32 = 32-sample chunks for the plain form too."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import build_variant  # noqa: E402


def chunk32(src):
    a = "    constexpr int kChunk = SLOW ? 16 : PF ? 32 : 64;"
    assert src.count(a) == 1
    return src.replace(a, "    constexpr int kChunk = SLOW ? 16 : 32;")


if __name__ == "__main__":
    print(build_variant("a32", chunk32))
