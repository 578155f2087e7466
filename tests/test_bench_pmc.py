"""bench.py's counter lookup: every bench kernel resolves to one entry of the committed counter summary.

Round 5's BENCH line lost `roofline.traffic` / `roofline.issue` because `k_encode_v4` grew template parameters and
the exact-string lookup stopped matching.  These CPU tests pin the lookup against the
committed `profiles/pmc_traffic.json` and the library stamp, without a GPU.
"""
import hashlib
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

SUMMARY = ROOT / "profiles" / "pmc_traffic.json"
LIB = ROOT / "flac_raster_amd" / "libflac_raster_amd.so"


def _summary():
    return json.loads(SUMMARY.read_text())


def test_every_bench_kernel_resolves_in_committed_summary():
    kernels = _summary()["kernels"]
    for name in bench.KERNEL_SYMBOL:
        sym = bench.resolve_symbol(kernels, name)
        assert sym is not None, f"{name}: {bench.KERNEL_SYMBOL[name]} not (uniquely) in {SUMMARY.name}"
        for field in ("bytes", "read_bytes", "write_bytes", "valu_insts"):
            assert field in kernels[sym], (name, field)


def test_step_kernels_present():
    kernels = _summary()["kernels"]
    for p in bench.STEP_KERNELS:
        assert any(k.startswith(p) for k in kernels), p


def test_resolve_symbol_prefix_rules():
    ks = {"frs::k_encode_v4<3, false, false, false>": {}, "frs::k_encode_v4<3, true, true, false>": {},
          "frs::k_analyze_v3<3, false, true, false>": {}, "frs::k_analyze_v3<3, true, false, false>": {}}
    assert bench.resolve_symbol(ks, "encode") == "frs::k_encode_v4<3, false, false, false>"
    assert bench.resolve_symbol(ks, "analyze") == "frs::k_analyze_v3<3, false, true, false>"
    assert bench.resolve_symbol({"frs::k_encode_v4<3, falsey>": {}}, "encode") is None
    two = {"frs::k_encode_v4<3, false, false, false>": {}, "frs::k_encode_v4<3, false, true, false>": {}}
    assert bench.resolve_symbol(two, "encode") is None  # ambiguous: never a guess


@pytest.mark.skipif(not LIB.exists(), reason="library not built")
def test_summary_stamp_matches_built_library_and_figures_flow():
    """The committed summary describes the library in the tree (the bench reports it only then), and the
    dominant kernel's traffic and the step traffic come out of the lookup."""
    d = _summary()
    if d.get("lib_sha256") != hashlib.sha256(LIB.read_bytes()).hexdigest():
        pytest.skip("library rebuilt since the counters were taken (a closing profile run restamps them)")
    px = d["pixels_per_launch"]
    enc = bench.pmc_for(str(SUMMARY), "encode", px, "bytes")
    assert enc and enc > 2 * px  # reads the band at least once
    st = bench.step_traffic_for(str(SUMMARY), px, 5.0)
    assert st and st["bytes"] >= enc
