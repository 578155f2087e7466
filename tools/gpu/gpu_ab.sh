#!/bin/bash
# A/B: bench each library variant under variants/ (FRS_LIB_PATH), 3 steps, no CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/ab/$n.log 2>&1 || exit 1
done
echo done
