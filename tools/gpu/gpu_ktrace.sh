#!/bin/bash
# rocprofv3 kernel-trace stats of one command: KT_CMD="python3 tools/sentinel_probe.py" -> gpurun_out/ktrace/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ktrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- ${KT_CMD} > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python3 tools/rocprof_summary.py $(find $O/kt -name "*kernel_stats.csv" | head -1) > $O/kernel_stats.md
cat $O/kernel_stats.md
