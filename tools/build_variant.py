#!/usr/bin/env python3
"""Build an experimental variant of libflac_raster_amd.so from a patched copy of frs_encode.hip.

Usage (from Python): build_variant(name, patch_fn) -> path of variants/lib<name>.so.  The other objects come
from the normal build (flac_raster_amd/csrc/*.o).  Select at run time with FRS_LIB_PATH=<path>.
"""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "flac_raster_amd" / "csrc"
OUT = ROOT / "variants"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-result",
         "-Wno-unused-value"]


def build_variant(name, patch_fn, src_name="frs_encode.hip", extra_flags=()):
    OUT.mkdir(exist_ok=True)
    src = (CSRC / src_name).read_text()
    new = patch_fn(src)
    if new == src and name not in ("base", "cur", "dbase") and not extra_flags:
        raise ValueError(f"variant {name}: patch did not apply")
    tmp = OUT / f"{name}_{src_name}"
    tmp.write_text(new)
    obj = OUT / f"{name}_{src_name}.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *FLAGS, *extra_flags, f"-I{CSRC}", "-c", "-o", str(obj),
                    str(tmp)], check=True)
    others = [str(p) for p in sorted(CSRC.glob("*.o")) if p.name != src_name.replace(".hip", ".o")]
    lib = OUT / f"lib{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(lib), str(obj),
                    *others], check=True)
    return lib
