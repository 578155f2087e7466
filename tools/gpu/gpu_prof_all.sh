#!/bin/bash
# kernel stats of a whole bench run (all legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/profall
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profall/raw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --queries 200 --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/profall/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/profall/bench.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/profall/bench.err; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/profall/raw -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/profall/kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/profall/kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:40]:
    print(f"{r['Name'][:90]:90s} n={r['Calls']:>6s} avg={float(r['AverageNs'])/1e3:9.1f}us tot={float(r['TotalDurationNs'])/1e6:8.2f}ms")
PY
