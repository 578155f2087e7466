#!/usr/bin/env python3
"""Round 6 selection-pass A/B: variants/libdold.so = the library with HEAD's frs_decode.hip (the per-dword 0xFF
branch in sel_masks_co, a lane scan per step in sel_emit_co), against the tree's build."""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import ROOT, build_variant  # noqa: E402

if __name__ == "__main__":
    rev = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
    old = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:flac_raster_amd/csrc/frs_decode.hip"], check=True,
                         capture_output=True, text=True).stdout
    print(build_variant("dold", lambda src: old, src_name="frs_decode.hip"))
