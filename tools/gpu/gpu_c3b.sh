#!/bin/bash
# C3 bench repeatability: three runs of 20 steps without the CPU baseline, then one with HIP-event profiling off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --height 16384 --width 16384 --steps 20 --warmup 3 --no-cpu --queries 0 >> gpurun_out/c3/rep.log 2>&1 || exit 1
done
echo done
