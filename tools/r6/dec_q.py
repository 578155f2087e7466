#!/usr/bin/env python3
"""Round 6 selection-queue variants (variants/lib<name>.so, FRS_LIB_PATH):
dq6 = the tree's k_sync_count with amdgpu_waves_per_eu(6, 8) (80 VGPRs, a 32-byte spill: 6 waves per SIMD)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import build_variant  # noqa: E402


def waves6(src):
    a = "__global__ void __launch_bounds__(kSelThreads) k_sync_count("
    assert src.count(a) == 1
    return src.replace(a, "__global__ void __launch_bounds__(kSelThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) k_sync_count(")


if __name__ == "__main__":
    print(build_variant("dq6", waves6, src_name="frs_decode.hip"))
