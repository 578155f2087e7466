"""The C-ABI library loads without a GPU and exports every function declared in include/*.h."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(frs_[a-z0-9_]+)\s*\(", txt))
    return names


@pytest.fixture(scope="module")
def lib():
    so = ROOT / "flac_raster_amd" / "libflac_raster_amd.so"
    if not so.exists():
        subprocess.run(["make", "-C", str(ROOT / "flac_raster_amd" / "csrc"), "-j8"], check=True)
    return ctypes.CDLL(str(so))


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_lists_every_symbol():
    from flac_raster_amd import _native
    assert set(_native.EXPORTS) == declared_functions()


def test_abi_version_and_no_device_behaviour(lib):
    from flac_raster_amd import _native
    L = _native.load_library()
    assert L.frs_abi_version() == 1
    if L.frs_device_count() == 0:
        with pytest.raises(_native.NativeUnavailable):
            _native.Context(0)


def test_desc_struct_layout_matches_header():
    """ctypes EncodeDesc must match frs_encode_desc (compiled offsets via a tiny C program)."""
    from flac_raster_amd._native import EncodeDesc
    src = ROOT / "include" / "flac_raster_amd.h"
    prog = f'''#include "{src}"
#include <stdio.h>
#include <stddef.h>
int main(void){{printf("%zu %zu %zu %zu\\n", sizeof(frs_encode_desc), offsetof(frs_encode_desc, norm_mode),
offsetof(frs_encode_desc, tile_begin), offsetof(frs_encode_desc, tile_end));return 0;}}'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "t.c"
        c.write_text(prog)
        subprocess.run(["gcc", "-o", str(Path(d) / "t"), str(c)], check=True)
        out = subprocess.run([str(Path(d) / "t")], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in out] == [ctypes.sizeof(EncodeDesc), EncodeDesc.norm_mode.offset,
                                     EncodeDesc.tile_begin.offset, EncodeDesc.tile_end.offset]
