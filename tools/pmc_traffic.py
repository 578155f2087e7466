#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 --pmc passes (run_counter_collection.csv).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [--label TEXT] [--pixels PIXELS_PER_LAUNCH] [--valu DIR]
                      [--lib PATH]

FETCH_SIZE and WRITE_SIZE are in KB per dispatch (summed over TCC instances here).  On gfx950 FETCH_SIZE
counts half the bytes of wide streaming reads, so it is doubled (MI355X_MICROARCH.md, "HBM [CDNA4]");
WRITE_SIZE is taken as is.  The JSON maps kernel short names to mean bytes per launch, and bench.py copies
the dominant kernel's figure into roofline.traffic.  --valu DIR (a `--pmc SQ_INSTS_VALU` pass) adds the mean
wave-level VALU instructions per launch, which bench.py turns into roofline.issue (VALU issue rate vs peak).
--lib PATH stamps the summary with the sha256 of the profiled library: bench.py uses the counters only when the
library it loaded has the same hash (counters of another build are never reported as this build's).
"""
import hashlib
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_dispatch(d, counter):
    vals = defaultdict(float)
    names = {}
    for f in Path(d).rglob("run_counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    out = defaultdict(list)
    for k, v in vals.items():
        out[names[k]].append(v)
    CALLS.update({k: len(v) for k, v in out.items()})
    return {k: sum(v) / len(v) for k, v in out.items()}


CALLS = {}  # dispatches per kernel in the last pass read


def main():
    fetch, write, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    label = sys.argv[sys.argv.index("--label") + 1] if "--label" in sys.argv else ""
    pixels = int(sys.argv[sys.argv.index("--pixels") + 1]) if "--pixels" in sys.argv else None
    fr = per_dispatch(fetch, "FETCH_SIZE")
    wr = per_dispatch(write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fr) | set(wr)):
        rd = 2 * fr.get(k, 0.0) * 1024
        wb = wr.get(k, 0.0) * 1024
        kernels[k] = {"read_bytes": rd, "write_bytes": wb, "bytes": rd + wb, "calls": CALLS.get(k, 0)}
    if "--valu" in sys.argv:
        for k, v in per_dispatch(sys.argv[sys.argv.index("--valu") + 1], "SQ_INSTS_VALU").items():
            kernels.setdefault(k, {})["valu_insts"] = v
    lib_sha = None
    if "--lib" in sys.argv:
        lib_sha = hashlib.sha256(Path(sys.argv[sys.argv.index("--lib") + 1]).read_bytes()).hexdigest()
    json.dump({"label": label, "pixels_per_launch": pixels, "fetch_correction": 2.0, "lib_sha256": lib_sha,
               "kernels": kernels}, open(dst, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k}: read {v.get('read_bytes', 0) / 1e9:.3f} GB write {v.get('write_bytes', 0) / 1e9:.3f} GB "
              f"valu {v.get('valu_insts', 0):.4g}")


if __name__ == "__main__":
    main()
