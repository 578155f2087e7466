#!/bin/bash
# Tile-stats scheduling A/B: GPU parity suite, then alternating bench runs of the overlapped stats with 2/4/8 groups,
# the fused variant (FRS_ABLATE 8192) and the serial kernels (FRS_ABLATE 4096), then a kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/fuse; mkdir -p gpurun_out/fuse
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fuse/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  for cfg in "0 2" "0 4" "0 8" "8192 4" "4096 4"; do
    set -- $cfg
    FRS_ABLATE=$1 FRS_STATS_GROUPS=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 >> gpurun_out/fuse/a$1_g$2.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fuse/kt -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/fuse/kt.log 2>&1 || exit 1
echo done
