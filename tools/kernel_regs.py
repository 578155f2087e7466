#!/usr/bin/env python3
"""VGPR / SGPR / LDS / scratch of the kernels in a built object (gfx950 code object inside the .hip_fatbin section).
usage: tools/kernel_regs.py [obj] [name-substring ...]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def kernel_regs(obj, subs=()):
    with tempfile.TemporaryDirectory() as td:
        fb, co = Path(td) / "fb.bin", Path(td) / "k.co"
        subprocess.run([LLVM / "llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", str(obj), str(Path(td) / "x.o")],
                       check=True)
        subprocess.run([LLVM / "clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([LLVM / "llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for b in notes.split("- .agpr_count"):
        nm = re.search(r"\.name:\s+(\S+)", b)
        if not nm or (subs and not any(s in nm.group(1) for s in subs)):
            continue

        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", b)
            return m.group(1) if m else "?"
        out.append((nm.group(1), g("vgpr_count"), g("sgpr_count"), g("group_segment_fixed_size"),
                    g("private_segment_fixed_size")))
    return out


def probe(src="flac_raster_amd/csrc/frs_encode.hip", out="/tmp/frs_probe.o"):
    """compile `src` with FRS_PROBE_I16 (int16 kernels only: a fraction of the full build time)"""
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-fno-fast-math", "-DFRS_PROBE_I16", "-c", "-o", out, src], check=True)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--probe":
        sys.argv[1] = probe()
    obj = sys.argv[1] if len(sys.argv) > 1 else "flac_raster_amd/csrc/frs_encode.o"
    for name, v, s, lds, priv in kernel_regs(obj, sys.argv[2:]):
        print(f"{name[:70]:70s} vgpr {v:>4} sgpr {s:>4} lds {lds:>6} scratch {priv}")
