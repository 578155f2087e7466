#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5tr/kt -o run -- python3 tools/gpu/c5_lat.py 40 > gpurun_out/c5tr/log.txt 2>&1 || { tail -5 gpurun_out/c5tr/log.txt; exit 1; }
f=$(find gpurun_out/c5tr/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if "decode" in r["Kernel_Name"] or "sync" in r["Kernel_Name"] or "span" in r["Kernel_Name"] or "chain" in r["Kernel_Name"]]
last = None
for r in sel[-24:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - last) / 1e3 if last else 0
    print(f'{r["Kernel_Name"][:40]:40s} dur {(e - s) / 1e3:8.1f} us  gap-before {gap:8.1f} us  grid {r.get("Grid_Size","")} wg {r.get("Workgroup_Size","")} lds {r.get("LDS_Block_Size", r.get("Lds_Size",""))} scratch {r.get("Scratch_Size","")}')
    last = e
PY
